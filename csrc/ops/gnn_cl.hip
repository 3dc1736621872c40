// Channel-lane GATv2 embedder kernels (H <= 32): the fast path behind gnn_forward/gnn_backward.
//
// Mapping (gfx950, wave64): one wave owns one graph at a time; lane = 32*half + c, where c is a
// feature channel and the two half-waves work on different nodes (v = 2r + half).  Feature maps
// live in LDS as [node][HP] rows (HP = H padded to a multiple of 4, zero-filled), so a lane reads
// a whole node/neighbour row with 16-byte broadcast loads while holding its own weight rows in
// VGPRs: the node linears become register FMA chains (2*HP FMAs per 16-byte load) instead of one
// LDS read per multiply-add.  Attention scores are per-message (lane = message) dot products over
// 16-byte row loads; softmax is per node; aggregation is per (node, channel).
//
// Numerics: fp32 throughout with the PyG GATv2Conv operation order (scores, max-shifted softmax
// + 1e-16, mean over in-degree).  Tested against gatv2_dense_reference (tests/test_gpu_ops.py).
#include <pybind11/pybind11.h>

#include "gnn_cl.h"

namespace py = pybind11;

namespace gsc {

// padded LDS parameter block: WlP[32][HP], WrP[32][HP], bl[32], br[32], att[32], bias[32]
template <int HP>
__host__ __device__ __forceinline__ int cl_pblock() { return 2 * 32 * HP + 4 * 32; }
__host__ __device__ __forceinline__ int cl_in_pad(int Fin) { return (Fin + 3) & ~3; }

// Stage every parameter block into the padded layout (zeros outside [H, Fi]).
template <int HP>
__device__ __forceinline__ void cl_stage_params(const ClArgs& a, float* P) {
  for (int b = 0; b < a.n_blocks; ++b) {
    const int Fi = b == 0 ? a.Fin : a.H;
    const float* src = a.params + cl_block_offset(b, a.Fin, a.H);
    float* dst = P + b * cl_pblock<HP>();
    for (int i = threadIdx.x; i < cl_pblock<HP>(); i += blockDim.x) {
      float v = 0.f;
      if (i < 2 * 32 * HP) {
        const int mat = i / (32 * HP), r = i - mat * 32 * HP, c = r / HP, k = r - c * HP;
        if (c < a.H && k < Fi) v = src[mat * (a.H * Fi + a.H) + c * Fi + k];
      } else {
        const int j = i - 2 * 32 * HP, which = j >> 5, c = j & 31;
        if (c < a.H) {
          // which: 0 bl, 1 br, 2 att, 3 bias
          const int off = which == 0 ? a.H * Fi : (which == 1 ? 2 * a.H * Fi + a.H : 2 * a.H * Fi + a.H * (which));
          v = src[off + c];
        }
      }
      dst[i] = v;
    }
  }
}

// One convolution. hin: [n][FIP] (FIP = Fi padded), outputs xl, xr: [n][HP], alpha [m], y: [n][HP].
template <int HP, int FIP>
__device__ __forceinline__ void cl_conv(const float* Pb, const ClTopo& T, const float* hin, float* xl, float* xr,
                                        float* alpha, float* y, bool relu, int lane) {
  const int half = lane >> 5, c = lane & 31;
  const float* WlP = Pb;
  const float* WrP = Pb + 32 * HP;
  const float* vec = Pb + 2 * 32 * HP;
  const int n = T.n, m = T.m;
  // ---- node linears: weight rows in VGPRs, node rows by 16-byte broadcast loads ----
  float wl[FIP], wr[FIP];
#pragma unroll
  for (int k4 = 0; k4 < FIP / 4; ++k4) {
    const float4 a4 = *reinterpret_cast<const float4*>(WlP + c * HP + 4 * k4);
    const float4 b4 = *reinterpret_cast<const float4*>(WrP + c * HP + 4 * k4);
    wl[4 * k4] = a4.x; wl[4 * k4 + 1] = a4.y; wl[4 * k4 + 2] = a4.z; wl[4 * k4 + 3] = a4.w;
    wr[4 * k4] = b4.x; wr[4 * k4 + 1] = b4.y; wr[4 * k4 + 2] = b4.z; wr[4 * k4 + 3] = b4.w;
  }
  const float blc = vec[c], brc = vec[32 + c];
  for (int v = half; v < n; v += 2) {
    float sl = blc, sr = brc;
    const float* hv = hin + v * FIP;
#pragma unroll
    for (int k4 = 0; k4 < FIP / 4; ++k4) {
      const float4 h4 = *reinterpret_cast<const float4*>(hv + 4 * k4);
      sl = fmaf(h4.x, wl[4 * k4], sl); sl = fmaf(h4.y, wl[4 * k4 + 1], sl);
      sl = fmaf(h4.z, wl[4 * k4 + 2], sl); sl = fmaf(h4.w, wl[4 * k4 + 3], sl);
      sr = fmaf(h4.x, wr[4 * k4], sr); sr = fmaf(h4.y, wr[4 * k4 + 1], sr);
      sr = fmaf(h4.z, wr[4 * k4 + 2], sr); sr = fmaf(h4.w, wr[4 * k4 + 3], sr);
    }
    if (c < HP) {
      xl[v * HP + c] = sl;
      xr[v * HP + c] = sr;
    }
  }
  cl_wave_sync();
  // ---- attention scores: lane = message ----
  float att[HP];
#pragma unroll
  for (int k4 = 0; k4 < HP / 4; ++k4) {
    const float4 t4 = *reinterpret_cast<const float4*>(vec + 64 + 4 * k4);
    att[4 * k4] = t4.x; att[4 * k4 + 1] = t4.y; att[4 * k4 + 2] = t4.z; att[4 * k4 + 3] = t4.w;
  }
  for (int q = lane; q < m; q += 64) {
    const float* xj = xl + T.isrc[q] * HP;
    const float* xi = xr + T.idst[q] * HP;
    float s = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < HP / 4; ++k4) {
      const float4 a4 = *reinterpret_cast<const float4*>(xj + 4 * k4);
      const float4 b4 = *reinterpret_cast<const float4*>(xi + 4 * k4);
      float z;
      z = a4.x + b4.x; s = fmaf(att[4 * k4], z > 0.f ? z : kClSlope * z, s);
      z = a4.y + b4.y; s = fmaf(att[4 * k4 + 1], z > 0.f ? z : kClSlope * z, s);
      z = a4.z + b4.z; s = fmaf(att[4 * k4 + 2], z > 0.f ? z : kClSlope * z, s);
      z = a4.w + b4.w; s = fmaf(att[4 * k4 + 3], z > 0.f ? z : kClSlope * z, s);
    }
    alpha[q] = s;
  }
  cl_wave_sync();
  // ---- segment softmax over each node's incoming messages ----
  for (int v = lane; v < n; v += 64) {
    const int q0 = T.iptr[v], q1 = T.iptr[v + 1];
    float mx = -INFINITY;
    for (int q = q0; q < q1; ++q) mx = fmaxf(mx, alpha[q]);
    float sum = 0.f;
    for (int q = q0; q < q1; ++q) {
      const float ex = __expf(alpha[q] - mx);
      alpha[q] = ex;
      sum += ex;
    }
    const float inv = 1.f / (sum + 1e-16f);
    for (int q = q0; q < q1; ++q) alpha[q] *= inv;
  }
  cl_wave_sync();
  // ---- aggregation (mean over in-degree) + bias (+ ReLU) ----
  const float biasc = vec[96 + c];
  for (int v = half; v < n; v += 2) {
    float acc = 0.f;
    for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) acc = fmaf(alpha[q], xl[T.isrc[q] * HP + (c < HP ? c : 0)], acc);
    float out = acc / T.deg[v] + biasc;
    if (relu) out = fmaxf(out, 0.f);
    if (c < HP) y[v * HP + c] = out;
  }
  cl_wave_sync();
}

template <int HP>
__host__ __device__ __forceinline__ int cl_fwd_per_wave(const ClArgs& a) {
  return 2 * a.NM * HP + 2 * a.NM * HP + ((a.M + 3) & ~3) + cl_topo_ints(a);
}

template <int HP>
__global__ __launch_bounds__(256) void gnn_cl_fwd_kernel(ClArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  cl_stage_params<HP>(a, lds);
  __syncthreads();
  constexpr int FIN_P = 4;  // encoder input padded to 4 (GSC: 3 node features)
  float* base = lds + a.n_blocks * cl_pblock<HP>() + wave * cl_fwd_per_wave<HP>(a);
  float* hA = base;
  float* hB = hA + a.NM * HP;
  float* xl = hB + a.NM * HP;
  float* xr = xl + a.NM * HP;
  float* al = xr + a.NM * HP;
  ClTopo T;
  cl_bind_topo(T, reinterpret_cast<int*>(al + ((a.M + 3) & ~3)), a);
  const int half = lane >> 5, c = lane & 31;
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    cl_load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    const float* xg = a.x + (long)g * a.P * a.Fin;
    for (int i = lane; i < n * FIN_P; i += 64) {
      const int v = i >> 2, k = i & 3;
      hA[i] = k < a.Fin ? xg[v * a.Fin + k] : 0.f;
    }
    cl_wave_sync();
    const float* hin = hA;
    float* hout = hB;
    for (int l = 0; l < a.L; ++l) {
      const float* Pb = lds + a.layer_of[l] * cl_pblock<HP>();
      const bool relu = l < a.L - 1 || a.L == 1;
      if (l == 0) cl_conv<HP, FIN_P>(Pb, T, hin, xl, xr, al, hout, relu, lane);
      else cl_conv<HP, HP>(Pb, T, hin, xl, xr, al, hout, relu, lane);
      float* tmp = const_cast<float*>(hin);
      hin = hout;
      hout = tmp;
    }
    // mean pool: each half sums its nodes, halves combined through LDS (xl is free now)
    float s = 0.f;
    for (int v = half; v < n; v += 2) s += hin[v * HP + (c < HP ? c : 0)];
    if (half == 1 && c < HP) xl[c] = s;
    cl_wave_sync();
    if (half == 0 && c < a.H) a.emb[(long)g * a.H + c] = (s + xl[c]) / (float)n;
    cl_wave_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
struct ClBwdLayout {
  int hin[kClMaxLayers], xl[kClMaxLayers], xr[kClMaxLayers], al[kClMaxLayers];
  int ylast, dy, dxl, dxr, da, acc, topo, per_wave;
};

template <int HP>
__host__ __device__ inline ClBwdLayout cl_bwd_layout(const ClArgs& a) {
  ClBwdLayout b{};
  int o = 0;
  const int M4 = (a.M + 3) & ~3;
  for (int l = 0; l < a.L; ++l) {
    const int FIP = l == 0 ? 4 : HP;
    b.hin[l] = o; o += a.NM * FIP;
    b.xl[l] = o; o += a.NM * HP;
    b.xr[l] = o; o += a.NM * HP;
    b.al[l] = o; o += M4;
  }
  b.ylast = o; o += a.NM * HP;
  b.dy = o; o += a.NM * HP;
  b.dxl = o; o += a.NM * HP;
  b.dxr = o; o += a.NM * HP;
  b.da = o; o += M4;
  b.acc = 0;
  b.topo = o; o += cl_topo_ints(a);
  if (o < a.n_blocks * cl_pblock<HP>()) o = a.n_blocks * cl_pblock<HP>();  // end-of-kernel gradient staging
  b.per_wave = (o + 3) & ~3;
  return b;
}

// Parameter-gradient accumulators of one parameter block, held in VGPRs for the whole
// grid-stride loop (lane c owns rows dWl[c,:], dWr[c,:] and the c-th bias/att entries; the two
// half-waves hold partial sums over different nodes and are combined once at the end).
template <int FIP>
struct ClGrad {
  float wl[FIP], wr[FIP];
  float bl, br, att, bias;
};

template <int FIP>
__device__ __forceinline__ void cl_grad_zero(ClGrad<FIP>& g) {
#pragma unroll
  for (int k = 0; k < FIP; ++k) { g.wl[k] = 0.f; g.wr[k] = 0.f; }
  g.bl = g.br = g.att = g.bias = 0.f;
}

// Backward of one convolution. dy: [n][HP] gradient of the conv output (after the ReLU mask);
// accumulates parameter gradients into G and, when need_dh, writes the input gradient into dh
// [n][FIP] (dh may alias dy: dy is fully consumed before dh is written).
template <int HP, int FIP>
__device__ __forceinline__ void cl_conv_bwd(const float* Pb, ClGrad<FIP>& G, const ClTopo& T, const float* hin,
                                            const float* xl, const float* xr, const float* al, const float* dy,
                                            float* dxl, float* dxr, float* da, float* dh, bool need_dh, int lane,
                                            ClClock& ck) {
  const int half = lane >> 5, c = lane & 31;
  const int cc = c < HP ? c : 0;
  const float* WlP = Pb;
  const float* WrP = Pb + 32 * HP;
  const float* vec = Pb + 2 * 32 * HP;
  const int n = T.n, m = T.m;
  for (int v = half; v < n; v += 2) G.bias += dy[v * HP + cc];
  // d alpha_q = (dy[i] . x_l[j]) / deg_i      (lane = message, target-sorted order)
  for (int q = lane; q < m; q += 64) {
    const int i = T.idst[q];
    const float* gi = dy + i * HP;
    const float* xj = xl + T.isrc[q] * HP;
    float s = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < HP / 4; ++k4) {
      const float4 a4 = *reinterpret_cast<const float4*>(gi + 4 * k4);
      const float4 b4 = *reinterpret_cast<const float4*>(xj + 4 * k4);
      s = fmaf(a4.x, b4.x, s); s = fmaf(a4.y, b4.y, s); s = fmaf(a4.z, b4.z, s); s = fmaf(a4.w, b4.w, s);
    }
    da[q] = s / T.deg[i];
  }
  cl_wave_sync();
  ck.mark(3);
  // softmax backward: de_q = alpha_q (da_q - sum_{q' -> i} alpha_q' da_q')   (contiguous per node)
  for (int v = lane; v < n; v += 64) {
    const int q0 = T.iptr[v], q1 = T.iptr[v + 1];
    float sad = 0.f;
    for (int q = q0; q < q1; ++q) sad = fmaf(al[q], da[q], sad);
    for (int q = q0; q < q1; ++q) da[q] = al[q] * (da[q] - sad);
  }
  cl_wave_sync();
  ck.mark(4);
  // d att_c = sum_q de_q lrelu(z_qc)   (lane = channel, halves split the messages)
  for (int q = half; q < m; q += 2) {
    float z = xl[T.isrc[q] * HP + cc] + xr[T.idst[q] * HP + cc];
    z = z > 0.f ? z : kClSlope * z;
    G.att = fmaf(da[q], z, G.att);
  }
  ck.mark(5);
  // dxl[v] = sum_{q: src=v} alpha_q dy[dst]/deg[dst] + dz_q ;  dxr[v] = sum_{q: dst=v} dz_q
  const float attc = vec[64 + c];
  for (int v = half; v < n; v += 2) {
    const float xlv = xl[v * HP + cc], xrv = xr[v * HP + cc];
    float sl = 0.f, sr = 0.f;
    for (int q = T.optr[v]; q < T.optr[v + 1]; ++q) {
      const int qi = T.oq[q];
      const int i = T.odst[q];
      const float z = xlv + xr[i * HP + cc];
      sl = fmaf(al[qi], dy[i * HP + cc] / T.deg[i], sl);
      sl = fmaf(da[qi] * attc, z > 0.f ? 1.f : kClSlope, sl);
    }
    for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) {
      const float z = xl[T.isrc[q] * HP + cc] + xrv;
      sr = fmaf(da[q] * attc, z > 0.f ? 1.f : kClSlope, sr);
    }
    if (c < HP) {
      dxl[v * HP + c] = sl;
      dxr[v * HP + c] = sr;
    }
  }
  cl_wave_sync();
  ck.mark(6);
  // weight gradients straight into the VGPR accumulators
  for (int v = half; v < n; v += 2) {
    const float el = dxl[v * HP + cc], er = dxr[v * HP + cc];
    G.bl += el;
    G.br += er;
    const float* hv = hin + v * FIP;
#pragma unroll
    for (int k4 = 0; k4 < FIP / 4; ++k4) {
      const float4 h4 = *reinterpret_cast<const float4*>(hv + 4 * k4);
      G.wl[4 * k4] = fmaf(el, h4.x, G.wl[4 * k4]); G.wl[4 * k4 + 1] = fmaf(el, h4.y, G.wl[4 * k4 + 1]);
      G.wl[4 * k4 + 2] = fmaf(el, h4.z, G.wl[4 * k4 + 2]); G.wl[4 * k4 + 3] = fmaf(el, h4.w, G.wl[4 * k4 + 3]);
      G.wr[4 * k4] = fmaf(er, h4.x, G.wr[4 * k4]); G.wr[4 * k4 + 1] = fmaf(er, h4.y, G.wr[4 * k4 + 1]);
      G.wr[4 * k4 + 2] = fmaf(er, h4.z, G.wr[4 * k4 + 2]); G.wr[4 * k4 + 3] = fmaf(er, h4.w, G.wr[4 * k4 + 3]);
    }
  }
  ck.mark(7);
  if (need_dh) {
    // dh[v,k] = sum_c dxl[v,c] Wl[c,k] + dxr[v,c] Wr[c,k]: lane k holds weight columns in VGPRs,
    // dxl/dxr rows arrive as 16-byte broadcasts
    const int k = c < FIP ? c : 0;
    float cl_[HP], cr_[HP];
#pragma unroll
    for (int c2 = 0; c2 < HP; ++c2) { cl_[c2] = WlP[c2 * HP + k]; cr_[c2] = WrP[c2 * HP + k]; }
    for (int v = half; v < n; v += 2) {
      const float* gl = dxl + v * HP;
      const float* gr = dxr + v * HP;
      float s = 0.f;
#pragma unroll
      for (int c4 = 0; c4 < HP / 4; ++c4) {
        const float4 a4 = *reinterpret_cast<const float4*>(gl + 4 * c4);
        const float4 b4 = *reinterpret_cast<const float4*>(gr + 4 * c4);
        s = fmaf(a4.x, cl_[4 * c4], s); s = fmaf(a4.y, cl_[4 * c4 + 1], s);
        s = fmaf(a4.z, cl_[4 * c4 + 2], s); s = fmaf(a4.w, cl_[4 * c4 + 3], s);
        s = fmaf(b4.x, cr_[4 * c4], s); s = fmaf(b4.y, cr_[4 * c4 + 1], s);
        s = fmaf(b4.z, cr_[4 * c4 + 2], s); s = fmaf(b4.w, cr_[4 * c4 + 3], s);
      }
      if (c < FIP) dh[v * FIP + c] = s;
    }
  }
  cl_wave_sync();
  ck.mark(8);
}

template <int FIP>
__device__ __forceinline__ void cl_grad_flush(const ClGrad<FIP>& G, float* row, int HP, int lane) {
  // combine the half-waves (lane l and l+32 hold partial sums of the same entries), lower half writes
  const int half = lane >> 5, c = lane & 31;
  float wl[FIP], wr[FIP];
#pragma unroll
  for (int k = 0; k < FIP; ++k) {
    wl[k] = G.wl[k] + __shfl_xor(G.wl[k], 32);
    wr[k] = G.wr[k] + __shfl_xor(G.wr[k], 32);
  }
  const float bl = G.bl + __shfl_xor(G.bl, 32), br = G.br + __shfl_xor(G.br, 32);
  const float at = G.att + __shfl_xor(G.att, 32), bi = G.bias + __shfl_xor(G.bias, 32);
  if (half == 0) {
#pragma unroll
    for (int k = 0; k < FIP; ++k) { row[c * HP + k] = wl[k]; row[32 * HP + c * HP + k] = wr[k]; }
    float* av = row + 2 * 32 * HP;
    av[c] = bl; av[32 + c] = br; av[64 + c] = at; av[96 + c] = bi;
  }
}

template <int HP, int NB, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void gnn_cl_bwd_kernel(ClArgs a,
                                                                                                ClBwdLayout bl) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  cl_stage_params<HP>(a, lds);
  float* W = lds + a.n_blocks * cl_pblock<HP>() + wave * bl.per_wave;
  __syncthreads();
  constexpr int FIN_P = 4;
  const int half = lane >> 5, c = lane & 31;
  const int cc = c < HP ? c : 0;
  ClGrad<FIN_P> GE;
  ClGrad<HP> GP;
  cl_grad_zero(GE);
  cl_grad_zero(GP);
  ClTopo T;
  cl_bind_topo(T, reinterpret_cast<int*>(W + bl.topo), a);
  float* dy = W + bl.dy;
  ClClock ck;
  ck.start(a.prof != nullptr);
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    cl_load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    const float* xg = a.x + (long)g * a.P * a.Fin;
    float* h0 = W + bl.hin[0];
    for (int i = lane; i < n * FIN_P; i += 64) {
      const int v = i >> 2, k = i & 3;
      h0[i] = k < a.Fin ? xg[v * a.Fin + k] : 0.f;
    }
    cl_wave_sync();
    // forward recompute (keeping every conv's input, x_l, x_r, alpha)
    for (int l = 0; l < a.L; ++l) {
      const float* Pb = lds + a.layer_of[l] * cl_pblock<HP>();
      float* y = (l + 1 < a.L) ? W + bl.hin[l + 1] : W + bl.ylast;
      const bool relu = l + 1 < a.L;  // the last conv's output stays pre-activation (ReLU mask below)
      if (l == 0) cl_conv<HP, FIN_P>(Pb, T, W + bl.hin[0], W + bl.xl[0], W + bl.xr[0], W + bl.al[0], y, relu, lane);
      else cl_conv<HP, HP>(Pb, T, W + bl.hin[l], W + bl.xl[l], W + bl.xr[l], W + bl.al[l], y, relu, lane);
    }
    ck.mark(1);
    // d emb -> dy of the last conv (mean pool), ReLU mask when the embedder has a single conv
    const float ge = c < a.H ? a.demb[(long)g * a.H + c] / (float)n : 0.f;
    for (int v = half; v < n; v += 2) {
      float d = ge;
      if (a.L == 1 && !(W[bl.ylast + v * HP + cc] > 0.f)) d = 0.f;
      if (c < HP) dy[v * HP + c] = d;
    }
    cl_wave_sync();
    for (int l = a.L - 1; l >= 0; --l) {
      const float* Pb = lds + a.layer_of[l] * cl_pblock<HP>();
      if (l == 0) {
        cl_conv_bwd<HP, FIN_P>(Pb, GE, T, W + bl.hin[0], W + bl.xl[0], W + bl.xr[0], W + bl.al[0], dy, W + bl.dxl,
                               W + bl.dxr, W + bl.da, dy, false, lane, ck);
      } else {
        cl_conv_bwd<HP, HP>(Pb, GP, T, W + bl.hin[l], W + bl.xl[l], W + bl.xr[l], W + bl.al[l], dy, W + bl.dxl,
                            W + bl.dxr, W + bl.da, dy, true, lane, ck);
        const float* post = W + bl.hin[l];  // post-ReLU output of conv l-1
        for (int v = half; v < n; v += 2)
          if (c < HP && !(post[v * HP + c] > 0.f)) dy[v * HP + c] = 0.f;
        cl_wave_sync();
        ck.mark(9);
      }
    }
  }
  if (ck.on && lane == 0)
    for (int k = 0; k < 12; ++k) atomicAdd(a.prof + k, ck.acc[k]);
  // per-wave accumulators -> LDS (reusing each wave's scratch) -> block sum -> partial row
  __syncthreads();
  float* accw = W;  // n_blocks * pblock floats fit inside the per-wave scratch (checked on the host)
  for (int i = lane; i < a.n_blocks * cl_pblock<HP>(); i += 64) accw[i] = 0.f;
  cl_wave_sync();
  cl_grad_flush<FIN_P>(GE, accw, HP, lane);
  if (NB > 1) cl_grad_flush<HP>(GP, accw + cl_pblock<HP>(), HP, lane);
  __syncthreads();
  const float* acc0 = lds + a.n_blocks * cl_pblock<HP>();
  for (int i = tid; i < a.n_params; i += blockDim.x) {
    int b = 0;
    while (b + 1 < a.n_blocks && i >= cl_block_offset(b + 1, a.Fin, a.H)) ++b;
    const int Fi = b == 0 ? a.Fin : a.H;
    const int r = i - cl_block_offset(b, a.Fin, a.H);
    const int WFi = a.H * Fi;
    int pidx;
    if (r < WFi) pidx = (r / Fi) * HP + (r % Fi);                                    // Wl
    else if (r < WFi + a.H) pidx = 2 * 32 * HP + (r - WFi);                           // bl
    else if (r < 2 * WFi + a.H) pidx = 32 * HP + ((r - WFi - a.H) / Fi) * HP + ((r - WFi - a.H) % Fi);  // Wr
    else pidx = 2 * 32 * HP + 32 * ((r - 2 * WFi - a.H) / a.H + 1) + ((r - 2 * WFi - a.H) % a.H);  // br/att/bias
    float s = 0.f;
    for (int w = 0; w < a.waves; ++w) s += acc0[(long)w * bl.per_wave + b * cl_pblock<HP>() + pidx];
    a.partials[(long)blockIdx.x * a.n_params + i] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// launchers (selected by gnn_forward / gnn_backward in gnn.hip when H <= 32 and Fin <= 4)
// ---------------------------------------------------------------------------------------------
template <int HP>
static void cl_launch_fwd(ClArgs a, hipStream_t st, int cus) {
  a.waves = 4;
  auto bytes = [&]() {
    return sizeof(float) * ((size_t)a.n_blocks * cl_pblock<HP>() + (size_t)a.waves * cl_fwd_per_wave<HP>(a));
  };
  while (a.waves > 1 && bytes() > 80 * 1024) a.waves--;
  const size_t lds = bytes();
  GSC_CHECK(lds <= 160 * 1024, "GNN forward working set exceeds LDS");
  if (lds > 65536)
    GSC_HIP_CHECK(hipFuncSetAttribute((const void*)gnn_cl_fwd_kernel<HP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int per_cu = (int)((160 * 1024) / lds);
  const int need = (a.B + a.waves - 1) / a.waves;
  const int cap = cus * (per_cu > 0 ? per_cu : 1);
  int grid = need < cap ? need : cap;
  hipLaunchKernelGGL(gnn_cl_fwd_kernel<HP>, dim3(grid > 0 ? grid : 1), dim3(64 * a.waves), lds, st, a);
  check_launch();
}

template <int HP>
static int cl_launch_bwd(ClArgs a, hipStream_t st, int cus, int max_rows) {
  ClBwdLayout bl{};
  a.waves = 4;
  size_t lds = 0;
  for (;;) {
    bl = cl_bwd_layout<HP>(a);
    lds = sizeof(float) * ((size_t)a.n_blocks * cl_pblock<HP>() + (size_t)a.waves * bl.per_wave);
    if (lds <= 80 * 1024 || a.waves == 1) break;
    a.waves--;
  }
  GSC_CHECK(lds <= 160 * 1024, "GNN backward working set exceeds LDS");
  // Register budget: 2 waves/SIMD (<= 256 VGPRs; a few spills for NB=2) measured 640 us vs 1179 us at
  // the unconstrained 287 VGPRs (1 wave/SIMD) for 25.6k Abilene graphs.  GSC_CL_WPE=1 restores the latter.
  static const int wpe = getenv("GSC_CL_WPE") ? atoi(getenv("GSC_CL_WPE")) : 2;
  const void* fn = a.n_blocks == 1 ? (wpe == 2 ? (const void*)gnn_cl_bwd_kernel<HP, 1, 2> : (const void*)gnn_cl_bwd_kernel<HP, 1, 1>)
                                   : (wpe == 2 ? (const void*)gnn_cl_bwd_kernel<HP, 2, 2> : (const void*)gnn_cl_bwd_kernel<HP, 2, 1>);
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int per_cu = (int)((160 * 1024) / lds);
  const int need = (a.B + a.waves - 1) / a.waves;
  const int cap = cus * (per_cu > 0 ? per_cu : 1);
  int grid = need < cap ? need : cap;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(reinterpret_cast<void (*)(ClArgs, ClBwdLayout)>(const_cast<void*>(fn)), dim3(grid),
                     dim3(64 * a.waves), lds, st, a, bl);
  check_launch();
  return grid;
}

// channel-lane path: H <= 32, <= 4 input features, encoder + at most one shared process block
bool gnn_cl_supported(int Fin, int H, int L, int n_blocks) {
  return Fin <= 4 && H <= 32 && L <= kClMaxLayers && n_blocks <= 2;
}

void gnn_cl_forward(const void* args_generic, uintptr_t stream, int cus) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 24) cl_launch_fwd<24>(a, stream_of(stream), cus);
  else cl_launch_fwd<32>(a, stream_of(stream), cus);
}

int gnn_cl_backward(const void* args_generic, uintptr_t stream, int cus, int max_rows) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 24) return cl_launch_bwd<24>(a, stream_of(stream), cus, max_rows);
  return cl_launch_bwd<32>(a, stream_of(stream), cus, max_rows);
}

}  // namespace gsc
