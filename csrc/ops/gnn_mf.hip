// MFMA GATv2 embedder kernels (gfx950): the default path behind gnn_forward/gnn_backward for
// GSC-sized graphs (H <= 32 channels, <= 32 nodes, <= 16 input features, encoder + one shared
// process block, every (source, target) message unique).
//
// One wave owns one graph at a time (persistent grid), and every dense product of a GATv2 layer
// runs on the matrix cores with v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32 accumulation):
//
//   node linears      X_l = h W_l^T + b_l       A = h rows (LDS image), B = W fragments
//   aggregation       Y = E X_l + bias          E[i][j] = alpha_{j->i} / deg_i (dense, LDS);
//                                               B = X_l straight from the linear's accumulators
//   weight gradients  dW += dX^T h              K = nodes; 4 x 16 accumulators live for the
//                                               whole grid-stride loop (deterministic, no atomics)
//   input gradients   dh = dX_l W_l + dX_r W_r  A = dX rows (LDS image), B = W^T fragments
//
//   message scatter   dX_r = S_dst G            S = one-hot [node][message] (per topology, global),
//                     dX_l = S_src G + E^T dy   G[q][c] = dL/dz of message q (bf16 LDS image);
//                                               dy straight from the previous dh accumulators
//
// The per-message rest of GATv2 runs on the VALU in fp32 with the PyG operation order, one
// message per lane: scores att . LeakyReLU(x_l[j] + x_r[i]); the per-target softmax max / sum as
// LDS atomics (ds_max_i32 on an order-preserving key, ds_add_f32); in the backward the softmax
// sum and G (lane = (message, quarter of the channels)).  No per-node loops: the dependent
// index -> data LDS chains of per-node VALU kernels are latency-bound.
//
// bf16 images: [node][k] rows (stride 40 bf16 = 80 B: conflict-free 16-byte fragment reads) and
// [k][node] (node-contiguous K operand of dW).  The backward keeps h (both images) and alpha per
// layer and recomputes x_l / x_r with 4 MFMAs when needed.
//
// Reference semantics: PyG GATv2Conv (reference src/rlsp/agents/models.py:10-53),
// as gatv2_dense_reference in gsc_amd/models/gnn.py.  Tests: tests/test_gpu_ops.py (bf16 tolerance).
#include <pybind11/pybind11.h>

#include <cstdlib>

#include "gnn_mf.h"

namespace gsc {

struct MfLayout {  // per-wave LDS offsets (bytes)
  int hR[kClMaxLayers], hT[kClMaxLayers], al[kClMaxLayers];
  int xl, xr, E, mx, sm, dy, U, da, topo, encW, encK, per_wave;
  int hTrows0, hTrows;  // rows of the [k][node] images: encoder input (Fin padded to 4), hidden (HPF)
  int blob;         // bytes of the per-layer images (hR, hT, alpha of every conv) = saved state per graph
  int NV, NVS, MS;  // node tile (16 | 32), [k][node] image stride, G^T image stride (bf16)
};

// per-wave copy of the graph's message list (target-sorted) and in-degrees
struct MfTopo {
  int *isrc, *idst;
  float* deg;
  int n, m, t;
};
__host__ __device__ __forceinline__ int mf_topo_bytes(const ClArgs& a) { return (2 * a.M + a.P) * 4; }
__device__ __forceinline__ void mf_bind_topo(MfTopo& T, char* base, const ClArgs& a) {
  T.isrc = reinterpret_cast<int*>(base);
  T.idst = T.isrc + a.M;
  T.deg = reinterpret_cast<float*>(T.idst + a.M);
  T.t = -1;
}
__device__ __forceinline__ void mf_load_topo(MfTopo& T, const ClArgs& a, int t, int lane) {
  T.n = a.nnodes[t];
  T.m = a.nmsgs[t];
  if (T.t == t) return;
  T.t = t;
  const long mo = (long)t * a.M;
  for (int i = lane; i < a.M; i += 64) {
    T.isrc[i] = a.in_src[mo + i];
    T.idst[i] = a.in_dst[mo + i];
  }
  for (int i = lane; i < a.P; i += 64) T.deg[i] = a.deg[(long)t * a.P + i];
  cl_wave_sync();
}

// Scores, per-target softmax (max and sum by LDS atomics), alpha (fp32, CSR order) and the dense
// bf16 aggregation matrix E[i][j] = alpha_{j->i} / deg_i.  mx / sm must be initialised.
template <int HPF>
__device__ __forceinline__ void mf_softmax(const float* vec, const MfTopo& T, const float* xl, const float* xr,
                                           float* alpha, int* mx, float* sm, __bf16* E, int NVS, bool write_e,
                                           int lane) {
  const int m = T.m;
  asm volatile("" ::: "memory");  // att is re-read from LDS per layer rather than held in VGPRs
  for (int q = lane; q < m; q += 64) {
    const int i = T.idst[q];
    const float* xj = xl + T.isrc[q] * mf_xs(HPF);
    const float* xi = xr + i * mf_xs(HPF);
    float s = 0.f;
#pragma unroll 2
    for (int k4 = 0; k4 < HPF / 4; ++k4) {
      const float4 a4 = *reinterpret_cast<const float4*>(xj + 4 * k4);
      const float4 b4 = *reinterpret_cast<const float4*>(xi + 4 * k4);
      const float4 t4 = *reinterpret_cast<const float4*>(vec + 64 + 4 * k4);
      float z;
      z = a4.x + b4.x; s = fmaf(t4.x, z > 0.f ? z : kClSlope * z, s);
      z = a4.y + b4.y; s = fmaf(t4.y, z > 0.f ? z : kClSlope * z, s);
      z = a4.z + b4.z; s = fmaf(t4.z, z > 0.f ? z : kClSlope * z, s);
      z = a4.w + b4.w; s = fmaf(t4.w, z > 0.f ? z : kClSlope * z, s);
    }
    alpha[q] = s;
    atomicMax(mx + i, mf_key(s));
  }
  cl_wave_sync();
  for (int q = lane; q < m; q += 64) {
    const int i = T.idst[q];
    const float ex = __expf(alpha[q] - mf_unkey(mx[i]));
    alpha[q] = ex;
    atomicAdd(sm + i, ex);
  }
  cl_wave_sync();
  for (int q = lane; q < m; q += 64) {
    const int i = T.idst[q];
    const float a = alpha[q] / (sm[i] + 1e-16f);
    alpha[q] = a;
    if (write_e) E[i * NVS + T.isrc[q]] = (__bf16)(a / T.deg[i]);
  }
  cl_wave_sync();
}

// Y = E X_l + bias on the matrix cores; X_l comes from the linear's accumulators (register i of
// k-step s is row 16s + 8(j>>2) + 4hh + (j&3) of X for element j, so E is read in that order).
__device__ __forceinline__ f32x16 mf_aggregate(const f32x16& xacc, const float* vec, const __bf16* E, int NV, int NVS,
                                               int lane) {
  const int r = lane & 31, hh = lane >> 5;
  const float bc = vec[96 + r];
  f32x16 y;
#pragma unroll
  for (int i = 0; i < 16; ++i) y[i] = bc;
  const __bf16* erow = E + (r < NV ? r : 0) * NVS + 4 * hh;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (s * 16 < NV) {
      bf16x8 xb;
#pragma unroll
      for (int j = 0; j < 8; ++j) xb[j] = (__bf16)xacc[8 * s + j];
      const bf16x4 e0 = *reinterpret_cast<const bf16x4*>(erow + 16 * s);
      const bf16x4 e1 = *reinterpret_cast<const bf16x4*>(erow + 16 * s + 8);
      const bf16x8 ea = __builtin_shufflevector(e0, e1, 0, 1, 2, 3, 4, 5, 6, 7);
      y = mf_mma(ea, xb, y);
    }
  }
  return y;
}

// One GATv2 layer.  MODE 0: hidden layer (ReLU output -> bf16 image(s)); 1: last layer, returns
// this lane's partial mean-pool sum; 2: last layer of the backward's recompute (alpha only).
template <int HPF, bool K2, int MODE, bool SAVE_T>
__device__ __forceinline__ float mf_layer(const MfW& w, const float* vec, const MfTopo& T, const __bf16* hin, float* xl,
                                          float* xr, float* alpha, int* mx, float* sm, __bf16* E, __bf16* hout,
                                          __bf16* houtT, int NV, int NVS, int H, int lane) {
  const int r = lane & 31, hh = lane >> 5;
  const int n = T.n;
  f32x16 al, ar;
  mf_linear<K2>(w, vec, hin, NV, lane, al, ar);
  mf_store_rows<HPF>(al, n, xl, lane);
  mf_store_rows<HPF>(ar, n, xr, lane);
  for (int v = lane; v < n; v += 64) {
    mx[v] = kMfKeyNegInf;
    sm[v] = 0.f;
  }
  cl_wave_sync();
  mf_softmax<HPF>(vec, T, xl, xr, alpha, mx, sm, E, NVS, MODE != 2, lane);
  if (MODE == 2) return 0.f;
  const f32x16 y = mf_aggregate(al, vec, E, NV, NVS, lane);
  if (MODE == 1) {
    const int nn = n - 4 * hh;
    float pool = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((i & 3) + 8 * (i >> 2) < nn) pool += y[i];
    return pool;
  }
  const int nn = n - 4 * hh;
  float o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = ((i & 3) + 8 * (i >> 2) < nn && r < H) ? fmaxf(y[i], 0.f) : 0.f;
  __bf16* hb = hout + 4 * hh * kMfRS + r;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ro = (i & 3) + 8 * (i >> 2);
    if (ro < 16 || NV > 16) hb[ro * kMfRS] = (__bf16)o[i];
  }
  if (SAVE_T && r < HPF) {
    __bf16* tb = houtT + r * NVS + 4 * hh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (8 * g < NV) {
        bf16x4 t;
        t[0] = (__bf16)o[4 * g]; t[1] = (__bf16)o[4 * g + 1]; t[2] = (__bf16)o[4 * g + 2]; t[3] = (__bf16)o[4 * g + 3];
        *reinterpret_cast<bf16x4*>(tb + 8 * g) = t;
      }
    }
  }
  cl_wave_sync();
  return 0.f;
}

// encoder input -> bf16 image(s); features beyond Fin and rows beyond n are zero.  Also clears
// the dense aggregation matrix (its non-edge entries must be zero for this graph's topology).
template <bool SAVE_T>
__device__ __forceinline__ void mf_load_x(const ClArgs& a, int g, int n, __bf16* hR, __bf16* hT, __bf16* E, int NV,
                                          int NVS, int lane) {
  mf_stage_input<SAVE_T>(a.x + (long)g * a.P * a.Fin, n, a.Fin, NV, hR, hT, NVS, (a.Fin + 3) & ~3, lane);
  for (int i = lane; i < NV * NVS / 8; i += 64) reinterpret_cast<uint4*>(E)[i] = make_uint4(0, 0, 0, 0);
  cl_wave_sync();
}

// NSETS = 2: a second parameter set (a.params2 -> a.emb2) on the same graphs in the same launch (the
// target actor's and the target critic's embedders of next_obs): one topology / input load per graph.
// (NSETS = 2 runs 8-wave workgroups: the second set's weights cost 9 KB of LDS per workgroup, which
// 4-wave workgroups would pay with a quarter fewer resident waves)
template <int HPF, bool K2, int NSETS>
__global__ __launch_bounds__(NSETS == 2 ? 512 : 256) __attribute__((amdgpu_waves_per_eu(4))) void gnn_mf_fwd_kernel(
    ClArgs a, MfLayout m) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // per parameter set: [bl br att bias per block][fragment sets: encoder, process]
  const int set_floats = mf_vec_floats(a.n_blocks) + 2 * kMfFragSet;
#pragma unroll
  for (int ws = 0; ws < NSETS; ++ws) {
    const float* P = ws == 0 ? a.params : a.params2;
    mf_stage_vec(a, lds + ws * set_floats, P);
    mf_stage_frags(a, reinterpret_cast<bf16x8*>(lds + ws * set_floats + mf_vec_floats(a.n_blocks)), 2, P);
  }
  __syncthreads();
  char* const W0 = reinterpret_cast<char*>(lds + NSETS * set_floats);
  int woff = wave * m.per_wave;
  MfTopo T;
  mf_bind_topo(T, W0 + woff + m.topo, a);
  const int half = lane >> 5, c = lane & 31;
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    asm volatile("" : "+v"(woff));  // see gnn_mf_bwd_kernel
    char* W = W0 + woff;
    __bf16* hA = reinterpret_cast<__bf16*>(W + m.hR[0]);
    __bf16* hB = reinterpret_cast<__bf16*>(W + m.hR[1]);
    float* xl = reinterpret_cast<float*>(W + m.xl);
    float* xr = reinterpret_cast<float*>(W + m.xr);
    float* al = reinterpret_cast<float*>(W + m.al[0]);
    __bf16* E = reinterpret_cast<__bf16*>(W + m.E);
    int* mx = reinterpret_cast<int*>(W + m.mx);
    float* sm = reinterpret_cast<float*>(W + m.sm);
    T.isrc = reinterpret_cast<int*>(W + m.topo);
    T.idst = T.isrc + a.M;
    T.deg = reinterpret_cast<float*>(T.idst + a.M);
    mf_load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    for (int ws = 0; ws < NSETS; ++ws) {
      const float* S0 = lds + ws * set_floats;
      const bf16x8* frags = reinterpret_cast<const bf16x8*>(S0 + mf_vec_floats(a.n_blocks));
      // the input image (and the cleared aggregation matrix) for this parameter set
      mf_load_x<false>(a, g, n, hA, nullptr, E, m.NV, m.NVS, lane);
      __bf16* hin = hA;
      __bf16* hout = hB;
      float pool = 0.f;
      for (int l = 0; l < a.L; ++l) {
        const float* vec = S0 + (l == 0 ? 0 : kMfVec);
        if (l + 1 < a.L) {
          if (l == 0)
            mf_layer<HPF, false, 0, false>(mf_frags(frags, 0, lane), vec, T, hin, xl, xr, al, mx, sm, E, hout, nullptr,
                                           m.NV, m.NVS, a.H, lane);
          else
            mf_layer<HPF, K2, 0, false>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, hout, nullptr,
                                        m.NV, m.NVS, a.H, lane);
          __bf16* t = hin;
          hin = hout;
          hout = t;
        } else {
          pool = mf_layer<HPF, K2, 1, false>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, nullptr,
                                             nullptr, m.NV, m.NVS, a.H, lane);
        }
      }
      pool += __shfl_xor(pool, 32);
      float* emb = ws == 0 ? a.emb : a.emb2;
      if (half == 0 && c < a.H) emb[(long)g * a.H + c] = pool / (float)n;
      cl_wave_sync();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
// Backward of one layer.  In: x_l / x_r fp32 rows and alpha of the layer, h^T (bf16), dy as an
// accumulator tile (dyt, rows = nodes, lane = channel) and as fp32 rows (LDS).  Out: parameter
// gradients accumulated (dW on the matrix cores, vectors per lane) and, when NEED_DH, dyt / dy
// rows of the layer below (dh masked by the ReLU of its output hin).
template <int HPF, bool K2, bool NEED_DH>
__device__ __forceinline__ void mf_layer_bwd(const ClArgs& a, const MfW* wT, const float* vec, MfVecGrad& G,
                                             float* gatt, f32x16& gl, f32x16& gr, const MfTopo& T, const float* xl,
                                             const float* xr, const float* al, const __bf16* hin, const __bf16* hT,
                                             f32x16& dyt, float* dy, float* da, float* ssum, __bf16* ET, __bf16* U,
                                             int NV, int NVS, int MS, int hTrows, int lane, ClClock& ck) {
  constexpr int CG = HPF / 4;
  const int r = lane & 31, hh = lane >> 5;
  const int n = T.n, m = T.m, nn = n - 4 * hh;
  G.bias += mf_colsum(dyt, nn);
  for (int i = lane; i < NV * NVS / 8; i += 64) reinterpret_cast<uint4*>(ET)[i] = make_uint4(0, 0, 0, 0);
  for (int v = lane; v < n; v += 64) ssum[v] = 0.f;
  cl_wave_sync();
  // p_q = alpha_q (dy[i] . x_l[j]) / deg_i ; ssum_i = sum_{q -> i} p_q ; E^T[j][i] = alpha_q / deg_i
  for (int q = lane; q < m; q += 64) {
    const int i = T.idst[q], j = T.isrc[q];
    const float* gi = dy + i * mf_xs(HPF);
    const float* xj = xl + j * mf_xs(HPF);
    float s = 0.f;
#pragma unroll 2
    for (int k4 = 0; k4 < HPF / 4; ++k4) {
      const float4 a4 = *reinterpret_cast<const float4*>(gi + 4 * k4);
      const float4 b4 = *reinterpret_cast<const float4*>(xj + 4 * k4);
      s = fmaf(a4.x, b4.x, s); s = fmaf(a4.y, b4.y, s); s = fmaf(a4.z, b4.z, s); s = fmaf(a4.w, b4.w, s);
    }
    const float ad = al[q] / T.deg[i];
    const float p = ad * s;
    da[q] = p;
    atomicAdd(ssum + i, p);
    ET[j * NVS + i] = (__bf16)ad;
  }
  cl_wave_sync();
  ck.mark(3);
  // de_q = p_q - alpha_q ssum_i ; per channel z = x_l[j] + x_r[i]:
  //   d att_c += de_q lrelu(z) ;  G[q][c] = de_q att_c lrelu'(z)   (stored as G^T[c][q], bf16)
  asm volatile("" ::: "memory");
  const int grp = lane & 3, c0 = grp * CG;
  for (int q = lane >> 2; q < m; q += 16) {
    const int i = T.idst[q], j = T.isrc[q];
    const float de = da[q] - al[q] * ssum[i];
#pragma unroll
    for (int k2 = 0; k2 < CG / 2; ++k2) {
      const int cx = c0 + 2 * k2;
      const float2 l2 = *reinterpret_cast<const float2*>(xl + j * mf_xs(HPF) + cx);
      const float2 r2 = *reinterpret_cast<const float2*>(xr + i * mf_xs(HPF) + cx);
      const float2 t2 = *reinterpret_cast<const float2*>(vec + 64 + cx);
      const float z0 = l2.x + r2.x, z1 = l2.y + r2.y;
      gatt[2 * k2] = fmaf(de, z0 > 0.f ? z0 : kClSlope * z0, gatt[2 * k2]);
      gatt[2 * k2 + 1] = fmaf(de, z1 > 0.f ? z1 : kClSlope * z1, gatt[2 * k2 + 1]);
      U[cx * MS + q] = (__bf16)(de * t2.x * (z0 > 0.f ? 1.f : kClSlope));
      U[(cx + 1) * MS + q] = (__bf16)(de * t2.y * (z1 > 0.f ? 1.f : kClSlope));
    }
  }
  cl_wave_sync();
  ck.mark(4);
  // dX_r = S_dst G ; dX_l = S_src G + E^T dy  (K = messages, then K = nodes with dy from registers)
  f32x16 dxl, dxr;
  mf_zero(dxl);
  mf_zero(dxr);
  {
    const __bf16* sd = reinterpret_cast<const __bf16*>(a.s_dst) + ((long)T.t * 32 + r) * a.MP + 8 * hh;
    const __bf16* ss = reinterpret_cast<const __bf16*>(a.s_src) + ((long)T.t * 32 + r) * a.MP + 8 * hh;
    const __bf16* gb = U + (r < HPF ? r : 0) * MS + 8 * hh;  // channels >= HPF: any finite data
    for (int s = 0; 16 * s < m; ++s) {
      const bf16x8 g8 = *reinterpret_cast<const bf16x8*>(gb + 16 * s);
      const bf16x8 d8 = *reinterpret_cast<const bf16x8*>(sd + 16 * s);
      const bf16x8 s8 = *reinterpret_cast<const bf16x8*>(ss + 16 * s);
      dxr = mf_mma(d8, g8, dxr);
      dxl = mf_mma(s8, g8, dxl);
    }
    const __bf16* erow = ET + (r < NV ? r : 0) * NVS;
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (16 * s < NV) dxl = mf_mma(mf_perm_frag(erow, s, hh), mf_pack(dyt, s), dxl);
  }
  G.bl += mf_colsum(dxl, nn);
  G.br += mf_colsum(dxr, nn);
  // dW[c][k] += sum_v dX[v][c] h[v][k]: dX^T as the A operand straight from the accumulators
  {
    const __bf16* hrow = hT + (r < hTrows ? r : 0) * NVS;  // columns k >= hTrows of dW are discarded
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (16 * s < NV) {
        const bf16x8 hb = mf_perm_frag(hrow, s, hh);
        gl = mf_mma(mf_pack(dxl, s), hb, gl);
        gr = mf_mma(mf_pack(dxr, s), hb, gr);
      }
    }
  }
  ck.mark(5);
  if (NEED_DH) {
    // dh[v][k] = sum_c dX_l[v][c] W_l[c][k] + dX_r[v][c] W_r[c][k] needs dX by rows: bf16 images
    // (reusing the G^T space), then the ReLU mask of hin
    cl_wave_sync();
    __bf16* xlR = U;
    __bf16* xrR = U + NV * kMfRS;
    {
      __bf16* bl = xlR + 4 * hh * kMfRS + r;
      __bf16* br = xrR + 4 * hh * kMfRS + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ro = (i & 3) + 8 * (i >> 2);
        if (ro < 16 || NV > 16) {
          bl[ro * kMfRS] = (__bf16)dxl[i];
          br[ro * kMfRS] = (__bf16)dxr[i];
        }
      }
    }
    cl_wave_sync();
    const MfW w = *wT;
    f32x16 acc;
    mf_zero(acc);
    const int vr = r < NV ? r : 0;
    acc = mf_mma(*reinterpret_cast<const bf16x8*>(xlR + vr * kMfRS + 8 * hh), w.l[0], acc);
    acc = mf_mma(*reinterpret_cast<const bf16x8*>(xrR + vr * kMfRS + 8 * hh), w.r[0], acc);
    if (K2) {
      acc = mf_mma(*reinterpret_cast<const bf16x8*>(xlR + vr * kMfRS + 16 + 8 * hh), w.l[1], acc);
      acc = mf_mma(*reinterpret_cast<const bf16x8*>(xrR + vr * kMfRS + 16 + 8 * hh), w.r[1], acc);
    }
    const __bf16* mb = hin + 4 * hh * kMfRS + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ro = (i & 3) + 8 * (i >> 2);
      dyt[i] = (ro < nn && (float)mb[(ro < 16 || NV > 16 ? ro : 0) * kMfRS] > 0.f) ? acc[i] : 0.f;
    }
    mf_store_rows<HPF>(dyt, n, dy, lane);
    cl_wave_sync();
    ck.mark(7);
  }
}

// WPE: waves per SIMD the register budget is sized for (2: 256 registers -- spills to scratch at
// H = 22; 1: 512 registers, no spills, one wave per SIMD)
template <int HPF, bool K2, bool LOADED, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void gnn_mf_bwd_kernel(ClArgs a, MfLayout m) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int CG = HPF / 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, half = hh, c = r;
  mf_stage_vec(a, lds);
  const bf16x8* frags = reinterpret_cast<const bf16x8*>(lds + mf_vec_floats(a.n_blocks));
  mf_stage_frags(a, reinterpret_cast<bf16x8*>(lds + mf_vec_floats(a.n_blocks)), 3);
  char* const W0 = reinterpret_cast<char*>(lds + mf_vec_floats(a.n_blocks) + 3 * kMfFragSet);
  char* W = W0 + wave * m.per_wave;
  // G^T columns beyond a graph's messages must hold finite values (they meet zeros of S)
  for (int i = lane; i < HPF * m.MS / 8; i += 64) reinterpret_cast<uint4*>(W + m.U)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  MfTopo T;
  mf_bind_topo(T, W + m.topo, a);
  // encoder dW (only k < Fin columns matter) accumulates in a small per-wave LDS image instead of
  // 32 more VGPRs live across the whole loop: [l|r][c < 32][k < encK]
  float* const encW = reinterpret_cast<float*>(W + m.encW);
  for (int i = lane; i < 2 * 32 * m.encK; i += 64) encW[i] = 0.f;
  f32x16 gPl, gPr;
  mf_zero(gPl);
  mf_zero(gPr);
  MfVecGrad GE{0.f, 0.f, 0.f}, GP{0.f, 0.f, 0.f};
  float gattE[CG], gattP[CG];
#pragma unroll
  for (int k = 0; k < CG; ++k) gattE[k] = gattP[k] = 0.f;
  const int NV = m.NV, NVS = m.NVS;
  int woff = wave * m.per_wave;
  // phase counters compiled out (a runtime-enabled clock pinned 26 registers for the whole loop and
  // pushed the kernel into scratch spills); gnn_bench's phase profile uses the channel-lane kernels
  ClClock ck;
  ck.start(false);
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    // opaque per-iteration base: stops LICM from materialising (and spilling) dozens of per-lane
    // LDS addresses for the whole loop; they are cheap to recompute
    asm volatile("" : "+v"(woff));
    W = W0 + woff;
    const int lane = mf_lane(), c = lane & 31, half = lane >> 5;
    float* xl = reinterpret_cast<float*>(W + m.xl);
    float* xr = reinterpret_cast<float*>(W + m.xr);
    float* dy = reinterpret_cast<float*>(W + m.dy);
    float* da = reinterpret_cast<float*>(W + m.da);
    __bf16* E = reinterpret_cast<__bf16*>(W + m.E);
    __bf16* U = reinterpret_cast<__bf16*>(W + m.U);
    int* mx = reinterpret_cast<int*>(W + m.mx);
    float* sm = reinterpret_cast<float*>(W + m.sm);
    T.isrc = reinterpret_cast<int*>(W + m.topo);
    T.idst = T.isrc + a.M;
    T.deg = reinterpret_cast<float*>(T.idst + a.M);
    mf_load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    if (LOADED) {
      // the forward saved every conv's input images and alpha: one bulk copy instead of a recompute,
      // as direct global -> LDS loads (1 KiB per wave instruction, all in flight together, no VGPRs)
      const char* src = reinterpret_cast<const char*>(a.blob) + (long)g * m.blob;
      for (int o = 0; o < m.blob; o += 1024)
        if (o + 16 * lane < m.blob)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + o + 16 * lane),
                                           (__attribute__((address_space(3))) void*)(W + o), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cl_wave_sync();
    } else {
      mf_load_x<true>(a, g, n, reinterpret_cast<__bf16*>(W + m.hR[0]), reinterpret_cast<__bf16*>(W + m.hT[0]), E, NV,
                      NVS, lane);
    }
    // forward recompute: keep each conv's input (both bf16 images) and alpha; the last conv's
    // output is not needed (its gradient comes from the mean pool)
    for (int l = 0; !LOADED && l < a.L; ++l) {
      const int lane = mf_lane();
      const float* vec = lds + (l == 0 ? 0 : kMfVec);
      const __bf16* hin = reinterpret_cast<const __bf16*>(W + m.hR[l]);
      float* al = reinterpret_cast<float*>(W + m.al[l]);
      __bf16* ho = l + 1 < a.L ? reinterpret_cast<__bf16*>(W + m.hR[l + 1]) : nullptr;
      __bf16* hoT = l + 1 < a.L ? reinterpret_cast<__bf16*>(W + m.hT[l + 1]) : nullptr;
      if (l + 1 == a.L)
        mf_layer<HPF, K2, 2, true>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, ho, hoT, NV, NVS,
                                   a.H, lane);
      else if (l == 0)
        mf_layer<HPF, false, 0, true>(mf_frags(frags, 0, lane), vec, T, hin, xl, xr, al, mx, sm, E, ho, hoT, NV, NVS,
                                      a.H, lane);
      else
        mf_layer<HPF, K2, 0, true>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, ho, hoT, NV, NVS,
                                   a.H, lane);
    }
    ck.mark(1);
    // d emb -> dy of the last conv (mean pool; the last conv has no ReLU), as a tile and as rows
    f32x16 dyt;
    {
      const float ge = c < a.H ? a.demb[(long)g * a.H + c] / (float)n : 0.f;
      const int nn = n - 4 * half;
#pragma unroll
      for (int i = 0; i < 16; ++i) dyt[i] = (i & 3) + 8 * (i >> 2) < nn ? ge : 0.f;
      mf_store_rows<HPF>(dyt, n, dy, lane);
    }
    for (int l = a.L - 1; l >= 0; --l) {
      const int lane = mf_lane(), r = lane & 31, hh = lane >> 5;
      const float* vec = lds + (l == 0 ? 0 : kMfVec);
      const __bf16* hin = reinterpret_cast<const __bf16*>(W + m.hR[l]);
      const __bf16* hT = reinterpret_cast<const __bf16*>(W + m.hT[l]);
      const float* al = reinterpret_cast<const float*>(W + m.al[l]);
      if (LOADED || l + 1 < a.L) {  // x_l / x_r of this conv (a recompute leaves the last conv's in place)
        f32x16 xa, xb;
        if (l == 0) mf_linear<false>(mf_frags(frags, 0, lane), vec, hin, NV, lane, xa, xb);
        else mf_linear<K2>(mf_frags(frags, 1, lane), vec, hin, NV, lane, xa, xb);
        mf_store_rows<HPF>(xa, n, xl, lane);
        mf_store_rows<HPF>(xb, n, xr, lane);
      }
      cl_wave_sync();
      ck.mark(2);
      if (l == 0) {
        f32x16 gEl, gEr;
        mf_zero(gEl);
        mf_zero(gEr);
        mf_layer_bwd<HPF, false, false>(a, nullptr, vec, GE, gattE, gEl, gEr, T, xl, xr, al, hin, hT, dyt, dy, da, sm,
                                        E, U, NV, NVS, m.MS, m.hTrows0, lane, ck);
        if (r < a.Fin) {
          float* el = reinterpret_cast<float*>(W + m.encW) + 4 * hh * m.encK + r;
          float* er = el + 32 * m.encK;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ro = (i & 3) + 8 * (i >> 2);
            el[ro * m.encK] += gEl[i];
            er[ro * m.encK] += gEr[i];
          }
        }
      } else {
        asm volatile("" ::: "memory");
        const MfW wT = mf_frags(frags, 2, lane);
        mf_layer_bwd<HPF, K2, true>(a, &wT, vec, GP, gattP, gPl, gPr, T, xl, xr, al, hin, hT, dyt, dy, da, sm, E, U,
                                    NV, NVS, m.MS, m.hTrows, lane, ck);
      }
    }
    cl_wave_sync();  // the next graph overwrites the images the last MFMAs read
  }
  if (ck.on && lane == 0)
    for (int k = 0; k < 12; ++k) atomicAdd(a.prof + k, ck.acc[k]);
  // per-wave gradients -> LDS image (each wave's own scratch) [block][Wl 32x32 | Wr 32x32 | bl br att bias]
  // -> block sum
  W = W0 + wave * m.per_wave;
  __syncthreads();
  float* img = reinterpret_cast<float*>(W);
  const float* ew = reinterpret_cast<const float*>(W + m.encW);  // beyond the image
  const int off1 = cl_block_offset(1, a.Fin, a.H);
  // one parameter block per pass: this wave's [Wl 32x32 | Wr 32x32 | bl br att bias] image, then the
  // block sum over waves into this workgroup's partial row
  for (int b = 0; b < 2; ++b) {
    __syncthreads();
    if (b == 0) {
      for (int i = lane; i < 2 * 32 * 32; i += 64) {
        const int mat = i >> 10, cc2 = (i >> 5) & 31, k = i & 31;
        img[i] = k < m.encK ? ew[(mat * 32 + cc2) * m.encK + k] : 0.f;
      }
    } else {
      float* b0 = img + 4 * hh * 32 + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ro = ((i & 3) + 8 * (i >> 2)) * 32;
        b0[ro] = gPl[i];
        b0[32 * 32 + ro] = gPr[i];
      }
    }
    const MfVecGrad& G = b == 0 ? GE : GP;
    const float bl = G.bl + __shfl_xor(G.bl, 32), br = G.br + __shfl_xor(G.br, 32);
    const float bi = G.bias + __shfl_xor(G.bias, 32);
    float* v = img + 2 * 32 * 32;
    if (half == 0) { v[c] = bl; v[32 + c] = br; v[96 + c] = bi; }
    // d att: lanes with the same channel group (lane & 3) hold partial sums over messages
#pragma unroll
    for (int k = 0; k < CG; ++k) {
      float e = b == 0 ? gattE[k] : gattP[k];
#pragma unroll
      for (int sh = 4; sh < 64; sh <<= 1) e += __shfl_xor(e, sh);
      const int ch = (lane & 3) * CG + k;
      if (lane < 4 && ch < 32) v[64 + ch] = e;
    }
    __syncthreads();
    const int Fi = b == 0 ? a.Fin : a.H;
    const int cnt = cl_block_size(Fi, a.H), first = b == 0 ? 0 : off1;
    for (int rr = tid; rr < cnt; rr += blockDim.x) {
      const int WFi = a.H * Fi;
      int idx;
      if (rr < WFi) idx = (rr / Fi) * 32 + rr % Fi;
      else if (rr < WFi + a.H) idx = 2 * 32 * 32 + (rr - WFi);
      else if (rr < 2 * WFi + a.H) idx = 32 * 32 + ((rr - WFi - a.H) / Fi) * 32 + (rr - WFi - a.H) % Fi;
      else idx = 2 * 32 * 32 + 32 * ((rr - 2 * WFi - a.H) / a.H + 1) + (rr - 2 * WFi - a.H) % a.H;
      float s = 0.f;
      for (int w = 0; w < a.waves; ++w) s += reinterpret_cast<const float*>(W0 + (long)w * m.per_wave)[idx];
      a.partials[(long)blockIdx.x * a.n_params + first + rr] = s;
    }
  }
}

// Forward that also saves, per graph, every conv's input images (hR, hT) and alpha in the
// backward's LDS arrangement (MfLayout::blob bytes), so the MFMA backward loads them instead of
// recomputing the forward.  Used when the embedder's parameters require gradients.
template <int HPF, bool K2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gnn_mf_fwd_save_kernel(ClArgs a,
                                                                                                   MfLayout m) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  mf_stage_vec(a, lds);
  const bf16x8* frags = reinterpret_cast<const bf16x8*>(lds + mf_vec_floats(a.n_blocks));
  mf_stage_frags(a, reinterpret_cast<bf16x8*>(lds + mf_vec_floats(a.n_blocks)), 2);
  __syncthreads();
  char* const W0 = reinterpret_cast<char*>(lds + mf_vec_floats(a.n_blocks) + 2 * kMfFragSet);
  int woff = wave * m.per_wave;
  MfTopo T;
  mf_bind_topo(T, W0 + woff + m.topo, a);
  const int half = lane >> 5, c = lane & 31;
  const int NV = m.NV, NVS = m.NVS;
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    asm volatile("" : "+v"(woff));  // see gnn_mf_bwd_kernel
    char* W = W0 + woff;
    float* xl = reinterpret_cast<float*>(W + m.xl);
    float* xr = reinterpret_cast<float*>(W + m.xr);
    __bf16* E = reinterpret_cast<__bf16*>(W + m.E);
    int* mx = reinterpret_cast<int*>(W + m.mx);
    float* sm = reinterpret_cast<float*>(W + m.sm);
    T.isrc = reinterpret_cast<int*>(W + m.topo);
    T.idst = T.isrc + a.M;
    T.deg = reinterpret_cast<float*>(T.idst + a.M);
    mf_load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    mf_load_x<true>(a, g, n, reinterpret_cast<__bf16*>(W + m.hR[0]), reinterpret_cast<__bf16*>(W + m.hT[0]), E, NV,
                    NVS, lane);
    float pool = 0.f;
    for (int l = 0; l < a.L; ++l) {
      const float* vec = lds + (l == 0 ? 0 : kMfVec);
      const __bf16* hin = reinterpret_cast<const __bf16*>(W + m.hR[l]);
      float* al = reinterpret_cast<float*>(W + m.al[l]);
      if (l + 1 < a.L) {
        __bf16* ho = reinterpret_cast<__bf16*>(W + m.hR[l + 1]);
        __bf16* hoT = reinterpret_cast<__bf16*>(W + m.hT[l + 1]);
        if (l == 0)
          mf_layer<HPF, false, 0, true>(mf_frags(frags, 0, lane), vec, T, hin, xl, xr, al, mx, sm, E, ho, hoT, NV,
                                        NVS, a.H, lane);
        else
          mf_layer<HPF, K2, 0, true>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, ho, hoT, NV, NVS,
                                     a.H, lane);
      } else {
        pool = mf_layer<HPF, K2, 1, false>(mf_frags(frags, 1, lane), vec, T, hin, xl, xr, al, mx, sm, E, nullptr,
                                           nullptr, NV, NVS, a.H, lane);
      }
    }
    pool += __shfl_xor(pool, 32);
    if (half == 0 && c < a.H) a.emb[(long)g * a.H + c] = pool / (float)n;
    cl_wave_sync();
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<char*>(a.blob) + (long)g * m.blob);
    for (int i = lane; i < m.blob / 16; i += 64) dst[i] = reinterpret_cast<const uint4*>(W)[i];
    cl_wave_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// kind 0: forward; 1: forward that saves its per-layer images (the blob region, laid out exactly as
// the backward's, then the forward's scratch -- none of the backward's buffers, so more waves fit);
// 2: backward
enum { kMfLayFwd = 0, kMfLaySave = 1, kMfLayBwd = 2 };
static MfLayout mf_layout(const ClArgs& a, int kind, int HPF) {
  const bool bwd = kind == kMfLayBwd, blob = kind != kMfLayFwd;
  MfLayout m{};
  m.NV = a.NM <= 16 ? 16 : 32;
  m.NVS = m.NV + 4;  // [k][node] rows: NV + 4 bf16 keeps b64 row reads / writes of 16-32 rows conflict-free
  m.MS = a.MP + 8;
  int o = 0;
  auto take = [&](int bytes) {
    const int at = o;
    o += (bytes + 15) & ~15;
    return at;
  };
  m.hTrows0 = (a.Fin + 3) & ~3;
  m.hTrows = HPF;
  const int hRb = m.NV * kMfRS * 2, M4b = ((a.M + 3) & ~3) * 4, fb = a.NM * mf_xs(HPF) * 4;
  const int Nb = ((a.NM + 3) & ~3) * 4;
  if (blob) {
    for (int l = 0; l < a.L; ++l) {
      m.hR[l] = take(hRb);
      m.hT[l] = take((l == 0 ? m.hTrows0 : m.hTrows) * m.NVS * 2);
      m.al[l] = take(M4b);
    }
    m.blob = o;
    if (bwd) {
      m.dy = take(fb);
      const int gt = HPF * m.MS * 2, dx = 2 * hRb;
      m.U = take(gt > dx ? gt : dx);
      m.da = take(M4b);
    }
  } else {
    m.hR[0] = take(hRb);
    m.hR[1] = take(hRb);
    m.al[0] = take(M4b);
  }
  m.xl = take(fb);
  m.xr = take(fb);
  m.E = take(m.NV * m.NVS * 2);
  m.mx = take(Nb);
  m.sm = take(Nb);
  m.topo = take(mf_topo_bytes(a));
  if (bwd) {
    if (o < kMfFlush * 4) o = kMfFlush * 4;  // end-of-kernel image (one parameter block per pass)
    m.encK = (a.Fin + 3) & ~3;
    m.encW = take(2 * 32 * m.encK * 4);  // outside the end-of-kernel image
  }
  m.per_wave = (o + 15) & ~15;
  return m;
}

bool gnn_mf_supported(int Fin, int H, int NM, int L, int n_blocks, const int* layer_of) {
  if (!(Fin <= 16 && H <= 32 && NM <= 32 && L >= 2 && L <= kClMaxLayers && n_blocks == 2)) return false;
  for (int l = 0; l < L; ++l)
    if ((l == 0) != (layer_of[l] == 0)) return false;
  return true;
}

template <int HPF, bool K2>
static void mf_launch_fwd(ClArgs a, hipStream_t st, int cus) {
  const bool save = a.blob != nullptr, two = a.params2 != nullptr;
  GSC_CHECK(!(save && two), "the saving forward takes one parameter set");
  const MfLayout m = mf_layout(a, save ? kMfLaySave : kMfLayFwd, HPF);
  a.waves = two ? 8 : 4;
  const size_t lds = sizeof(float) * (two ? 2 : 1) * (mf_vec_floats(a.n_blocks) + 2 * kMfFragSet) +
                     (size_t)a.waves * m.per_wave;
  GSC_CHECK(lds <= 160 * 1024, "GNN (MFMA) forward working set exceeds LDS");
  const void* fn = save ? (const void*)gnn_mf_fwd_save_kernel<HPF, K2>
                        : (two ? (const void*)gnn_mf_fwd_kernel<HPF, K2, 2> : (const void*)gnn_mf_fwd_kernel<HPF, K2, 1>);
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu * a.waves > 16) per_cu = 16 / a.waves;  // 4 waves/SIMD (VGPR budget)
  const int need = (a.B + a.waves - 1) / a.waves;
  const int cap = cus * (per_cu > 0 ? per_cu : 1);
  const int grid = need < cap ? need : cap;
  if (save)
    hipLaunchKernelGGL((gnn_mf_fwd_save_kernel<HPF, K2>), dim3(grid > 0 ? grid : 1), dim3(64 * a.waves), lds, st, a, m);
  else if (two)
    hipLaunchKernelGGL((gnn_mf_fwd_kernel<HPF, K2, 2>), dim3(grid > 0 ? grid : 1), dim3(64 * a.waves), lds, st, a, m);
  else
    hipLaunchKernelGGL((gnn_mf_fwd_kernel<HPF, K2, 1>), dim3(grid > 0 ? grid : 1), dim3(64 * a.waves), lds, st, a, m);
  check_launch();
}

template <int HPF, bool K2>
static int mf_launch_bwd(ClArgs a, hipStream_t st, int cus, int max_rows) {
  static const int wpe = getenv("GSC_GNN_BWD_WPE") ? atoi(getenv("GSC_GNN_BWD_WPE")) : 2;  // measured: 336 vs 469 us (WPE 1)
  GSC_CHECK(a.s_dst != nullptr && a.s_src != nullptr && a.MP >= a.M && a.MP % 16 == 0,
            "MFMA GNN backward needs the one-hot message matrices (GraphSet.s_dst / s_src)");
  const MfLayout m = mf_layout(a, kMfLayBwd, HPF);
  a.waves = 4;
  size_t lds = 0;
  for (;;) {
    lds = sizeof(float) * (mf_vec_floats(a.n_blocks) + 3 * kMfFragSet) + (size_t)a.waves * m.per_wave;
    if (lds <= 80 * 1024 || a.waves == 1) break;
    a.waves--;
  }
  GSC_CHECK(lds <= 160 * 1024, "GNN (MFMA) backward working set exceeds LDS");
  const bool loaded = a.blob != nullptr;
  const void* fns[4] = {(const void*)gnn_mf_bwd_kernel<HPF, K2, true, 1>, (const void*)gnn_mf_bwd_kernel<HPF, K2, false, 1>,
                        (const void*)gnn_mf_bwd_kernel<HPF, K2, true, 2>, (const void*)gnn_mf_bwd_kernel<HPF, K2, false, 2>};
  const void* fn = fns[(wpe == 2 ? 2 : 0) + (loaded ? 0 : 1)];
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu * a.waves > 4 * wpe) per_cu = 4 * wpe / a.waves;  // WPE waves/SIMD (register budget)
  if (per_cu < 1) per_cu = 1;
  const int need = (a.B + a.waves - 1) / a.waves;
  const int cap = cus * (per_cu > 0 ? per_cu : 1);
  int grid = need < cap ? need : cap;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  if (wpe == 2) {
    if (loaded) hipLaunchKernelGGL((gnn_mf_bwd_kernel<HPF, K2, true, 2>), dim3(grid), dim3(64 * a.waves), lds, st, a, m);
    else hipLaunchKernelGGL((gnn_mf_bwd_kernel<HPF, K2, false, 2>), dim3(grid), dim3(64 * a.waves), lds, st, a, m);
  } else {
    if (loaded) hipLaunchKernelGGL((gnn_mf_bwd_kernel<HPF, K2, true, 1>), dim3(grid), dim3(64 * a.waves), lds, st, a, m);
    else hipLaunchKernelGGL((gnn_mf_bwd_kernel<HPF, K2, false, 1>), dim3(grid), dim3(64 * a.waves), lds, st, a, m);
  }
  check_launch();
  return grid;
}

void gnn_mf_forward(const void* args_generic, uintptr_t stream, int cus) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 16) mf_launch_fwd<24, false>(a, stream_of(stream), cus);
  else if (a.H <= 24) mf_launch_fwd<24, true>(a, stream_of(stream), cus);
  else mf_launch_fwd<32, true>(a, stream_of(stream), cus);
}

int gnn_mf_saved_bytes(const void* args_generic) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  return mf_layout(a, kMfLayBwd, a.H <= 24 ? 24 : 32).blob;
}

int gnn_mf_backward(const void* args_generic, uintptr_t stream, int cus, int max_rows) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 16) return mf_launch_bwd<24, false>(a, stream_of(stream), cus, max_rows);
  if (a.H <= 24) return mf_launch_bwd<24, true>(a, stream_of(stream), cus, max_rows);
  return mf_launch_bwd<32, true>(a, stream_of(stream), cus, max_rows);
}

}  // namespace gsc
