// Fused GATv2 embedder (reference models.py:10-53 on PyG GATv2Conv, aggr='mean') for gfx950.
//
// One 64-lane wave owns one graph at a time (persistent grid-stride loop); a workgroup holds up
// to four waves that share the embedder weights staged once in LDS.  Everything for a graph —
// node features, x_l/x_r, per-message attention, softmax, aggregation, ReLU, mean-pool — lives in
// LDS, as do the graph's message tables (copied per wave when the topology changes), so inner
// loops never wait on global memory.  The whole 3-convolution embedder costs one pass over the
// [B, n_pad, F] input.
//
// Backward recomputes the forward for its graph in LDS (cheaper than round-tripping activations
// through HBM), backpropagates through pool -> conv stack, and accumulates weight gradients in a
// per-wave LDS accumulator (each element owned by one lane: no atomics, deterministic).  Waves are
// reduced within the workgroup; workgroup partial rows are reduced by a parallel column-sum kernel.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <vector>

#include "../common.h"

namespace py = pybind11;

namespace gsc {

constexpr int kGnnMaxLayers = 16;
constexpr float kNegSlope = 0.2f;

struct GnnArgs {
  const float* params;
  const float* x;          // [B, P, Fin]
  const int32_t* topo;     // [B]
  const int32_t* src;      // [T, M]
  const int32_t* dst;      // [T, M]
  const int32_t* in_ptr;   // [T, P+1]
  const int32_t* in_msg;   // [T, M]
  const int32_t* out_ptr;  // [T, P+1]
  const int32_t* out_msg;  // [T, M]
  const float* deg;        // [T, P]
  const int32_t* nnodes;   // [T]
  const int32_t* nmsgs;    // [T]
  float* emb;              // [B, H]
  const float* demb;       // [B, H]
  float* partials;         // [grid, n_params]
  int B, P, Fin, H, L, M, NM, n_params, waves;
  int layer_of[kGnnMaxLayers];
  unsigned long long* prof;  // optional per-phase cycle counters (gnn_set_profile)
};

// Per-phase cycle accounting for the profiling instantiation (wave-uniform, s_memtime based).
template <bool PROF>
struct PhaseClock {
  unsigned long long last = 0, acc[12] = {};
  __device__ __forceinline__ void start() { if (PROF) last = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void mark(int k) {
    if (PROF) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
  __device__ __forceinline__ void flush(unsigned long long* out, int lane) {
    if (PROF && out && lane == 0)
      for (int k = 0; k < 12; ++k) atomicAdd(out + k, acc[k]);
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ __forceinline__ int block_size(int Fi, int H) { return 2 * H * Fi + 4 * H; }
__host__ __device__ __forceinline__ int block_offset(int b, int Fin, int H) {
  return b == 0 ? 0 : block_size(Fin, H) + (b - 1) * block_size(H, H);
}

// exact idx / d for the small index ranges used here (idx < 2^16, d < 2^8)
__device__ __forceinline__ int fdiv(int idx, float inv) { return (int)(((float)idx + 0.5f) * inv); }

struct LayerP {
  const float *Wl, *bl, *Wr, *br, *att, *bias;
  int Fi, off;
};

__device__ __forceinline__ LayerP layer_params(const float* P, const GnnArgs& a, int l) {
  const int b = a.layer_of[l];
  const int Fi = b == 0 ? a.Fin : a.H;
  const int H = a.H;
  LayerP p;
  p.off = block_offset(b, a.Fin, H);
  p.Fi = Fi;
  p.Wl = P + p.off;
  p.bl = p.Wl + H * Fi;
  p.Wr = p.bl + H;
  p.br = p.Wr + H * Fi;
  p.att = p.br + H;
  p.bias = p.att + H;
  return p;
}

// Per-wave LDS copy of one topology's message tables.
struct Topo {
  int* src;
  int* dst;
  int* iptr;
  int* imsg;
  int* optr;
  int* omsg;
  float* deg;
  int n, m, t;
};

__host__ __device__ __forceinline__ int topo_ints(const GnnArgs& a) { return 4 * a.M + 2 * (a.P + 1) + a.P; }

__device__ __forceinline__ void bind_topo(Topo& T, int* base, const GnnArgs& a) {
  T.src = base;
  T.dst = T.src + a.M;
  T.imsg = T.dst + a.M;
  T.omsg = T.imsg + a.M;
  T.iptr = T.omsg + a.M;
  T.optr = T.iptr + a.P + 1;
  T.deg = reinterpret_cast<float*>(T.optr + a.P + 1);
  T.t = -1;
}

__device__ __forceinline__ void load_topo(Topo& T, const GnnArgs& a, int t, int lane) {
  T.n = a.nnodes[t];
  T.m = a.nmsgs[t];
  if (T.t == t) return;
  T.t = t;
  const long mo = (long)t * a.M, po = (long)t * (a.P + 1);
  for (int i = lane; i < a.M; i += 64) {
    T.src[i] = a.src[mo + i];
    T.dst[i] = a.dst[mo + i];
    T.imsg[i] = a.in_msg[mo + i];
    T.omsg[i] = a.out_msg[mo + i];
  }
  for (int i = lane; i <= a.P; i += 64) {
    T.iptr[i] = a.in_ptr[po + i];
    T.optr[i] = a.out_ptr[po + i];
  }
  for (int i = lane; i < a.P; i += 64) T.deg[i] = a.deg[(long)t * a.P + i];
  wave_sync();
}

// One GATv2 convolution for one graph, all operands in LDS.  hin [n, Fi] -> y [n, H] (pre-activation);
// also leaves x_l, x_r and the attention weights alpha [m] in the given buffers.
__device__ __forceinline__ void gat_conv(const LayerP& p, const GnnArgs& a, const Topo& T, const float* hin, float* xl,
                                         float* xr, float* alpha, float* y, int lane, float invH) {
  const int H = a.H, Fi = p.Fi, n = T.n, m = T.m;
  for (int idx = lane; idx < n * H; idx += 64) {
    const int v = fdiv(idx, invH), c = idx - v * H;
    float sl = p.bl[c], sr = p.br[c];
    const float* hv = hin + v * Fi;
    const float* wl = p.Wl + c * Fi;
    const float* wr = p.Wr + c * Fi;
#pragma unroll 4
    for (int k = 0; k < Fi; ++k) {
      const float h = hv[k];
      sl = fmaf(h, wl[k], sl);
      sr = fmaf(h, wr[k], sr);
    }
    xl[idx] = sl;
    xr[idx] = sr;
  }
  wave_sync();
  for (int q = lane; q < m; q += 64) {
    const float* xj = xl + T.src[q] * H;
    const float* xi = xr + T.dst[q] * H;
    float s = 0.f;
#pragma unroll 4
    for (int c = 0; c < H; ++c) {
      float z = xj[c] + xi[c];
      z = z > 0.f ? z : kNegSlope * z;
      s = fmaf(p.att[c], z, s);
    }
    alpha[q] = s;
  }
  wave_sync();
  for (int v = lane; v < n; v += 64) {
    const int q0 = T.iptr[v], q1 = T.iptr[v + 1];
    float mx = -INFINITY;
    for (int q = q0; q < q1; ++q) mx = fmaxf(mx, alpha[T.imsg[q]]);
    float sum = 0.f;
    for (int q = q0; q < q1; ++q) {
      const int mi = T.imsg[q];
      const float ex = __expf(alpha[mi] - mx);
      alpha[mi] = ex;
      sum += ex;
    }
    const float inv = 1.f / (sum + 1e-16f);
    for (int q = q0; q < q1; ++q) alpha[T.imsg[q]] *= inv;
  }
  wave_sync();
  for (int idx = lane; idx < n * H; idx += 64) {
    const int v = fdiv(idx, invH), c = idx - v * H;
    float acc = 0.f;
    for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) {
      const int mi = T.imsg[q];
      acc = fmaf(alpha[mi], xl[T.src[mi] * H + c], acc);
    }
    y[idx] = acc / T.deg[v] + p.bias[c];
  }
  wave_sync();
}

__device__ __forceinline__ bool relu_after(const GnnArgs& a, int l) { return l < a.L - 1 || a.L == 1; }

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ int fwd_per_wave(const GnnArgs& a) {
  const int Hm = a.H > a.Fin ? a.H : a.Fin;
  return ((2 * a.NM * Hm + 2 * a.NM * a.H + a.M + topo_ints(a)) + 3) & ~3;
}

__global__ __launch_bounds__(256) void gnn_fwd_kernel(GnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < a.n_params; i += blockDim.x) lds[i] = a.params[i];
  __syncthreads();
  const int Hm = a.H > a.Fin ? a.H : a.Fin;
  float* hA = lds + ((a.n_params + 3) & ~3) + wave * fwd_per_wave(a);
  float* hB = hA + a.NM * Hm;
  float* xl = hB + a.NM * Hm;
  float* xr = xl + a.NM * a.H;
  float* al = xr + a.NM * a.H;
  Topo T;
  bind_topo(T, reinterpret_cast<int*>(al + a.M), a);
  const int H = a.H;
  const float invH = 1.f / (float)H;
  for (int g = blockIdx.x * a.waves + wave; g < a.B; g += gridDim.x * a.waves) {
    load_topo(T, a, a.topo[g], lane);
    const int n = T.n;
    const float* xg = a.x + (long)g * a.P * a.Fin;
    for (int i = lane; i < n * a.Fin; i += 64) hA[i] = xg[i];
    wave_sync();
    float* hin = hA;
    float* hout = hB;
    for (int l = 0; l < a.L; ++l) {
      const LayerP p = layer_params(lds, a, l);
      gat_conv(p, a, T, hin, xl, xr, al, hout, lane, invH);
      if (relu_after(a, l)) {
        for (int i = lane; i < n * H; i += 64) hout[i] = fmaxf(hout[i], 0.f);
        wave_sync();
      }
      float* tmp = hin;
      hin = hout;
      hout = tmp;
    }
    const float inv_n = 1.f / (float)n;
    for (int c = lane; c < H; c += 64) {
      float s = 0.f;
      for (int v = 0; v < n; ++v) s += hin[v * H + c];
      a.emb[(long)g * H + c] = s * inv_n;
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// backward (recompute forward per graph, then reverse)
// ---------------------------------------------------------------------------------------------
struct BwdLayout {
  int hin[kGnnMaxLayers], xl[kGnnMaxLayers], xr[kGnnMaxLayers], al[kGnnMaxLayers];
  int ylast, dy, dxl, dxr, da, acc, topo, per_wave;
};

__host__ __device__ inline BwdLayout bwd_layout(const GnnArgs& a) {
  BwdLayout b{};
  int o = 0;
  for (int l = 0; l < a.L; ++l) {
    const int Fi = a.layer_of[l] == 0 ? a.Fin : a.H;
    b.hin[l] = o; o += a.NM * Fi;
    b.xl[l] = o; o += a.NM * a.H;
    b.xr[l] = o; o += a.NM * a.H;
    b.al[l] = o; o += a.M;
  }
  b.ylast = o; o += a.NM * a.H;  // pre-activation of the last conv (its ReLU mask when L == 1)
  const int Hm = a.H > a.Fin ? a.H : a.Fin;
  b.dy = o; o += a.NM * Hm;
  b.dxl = o; o += a.NM * a.H;
  b.dxr = o; o += a.NM * a.H;
  b.da = o; o += a.M;
  b.acc = o; o += a.n_params;
  b.topo = o; o += topo_ints(a);
  b.per_wave = (o + 3) & ~3;
  return b;
}

template <bool PROF>
__global__ __launch_bounds__(256) void gnn_bwd_kernel(GnnArgs a, BwdLayout bl) {
  PhaseClock<PROF> clk;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < a.n_params; i += blockDim.x) lds[i] = a.params[i];
  float* W = lds + ((a.n_params + 3) & ~3) + wave * bl.per_wave;
  float* acc = W + bl.acc;
  for (int i = lane; i < a.n_params; i += 64) acc[i] = 0.f;
  __syncthreads();
  const int H = a.H;
  const float invH = 1.f / (float)H;
  float* dy = W + bl.dy;
  float* dxl = W + bl.dxl;
  float* dxr = W + bl.dxr;
  float* da = W + bl.da;
  Topo T;
  bind_topo(T, reinterpret_cast<int*>(W + bl.topo), a);
  clk.start();
  for (int gi = blockIdx.x * a.waves + wave; gi < a.B; gi += gridDim.x * a.waves) {
    load_topo(T, a, a.topo[gi], lane);
    const int n = T.n, m = T.m;
    clk.mark(0);
    // ---- forward recompute ----
    const float* xg = a.x + (long)gi * a.P * a.Fin;
    for (int i = lane; i < n * a.Fin; i += 64) W[bl.hin[0] + i] = xg[i];
    wave_sync();
    for (int l = 0; l < a.L; ++l) {
      const LayerP p = layer_params(lds, a, l);
      float* y = (l + 1 < a.L) ? W + bl.hin[l + 1] : W + bl.ylast;
      gat_conv(p, a, T, W + bl.hin[l], W + bl.xl[l], W + bl.xr[l], W + bl.al[l], y, lane, invH);
      if (l + 1 < a.L) {
        for (int i = lane; i < n * H; i += 64) y[i] = fmaxf(y[i], 0.f);
        wave_sync();
      }
    }
    clk.mark(1);
    // ---- d emb -> dy of the last conv ----
    const float inv_n = 1.f / (float)n;
    for (int idx = lane; idx < n * H; idx += 64) {
      const int v = fdiv(idx, invH), c = idx - v * H;
      dy[idx] = a.demb[(long)gi * H + c] * inv_n;
    }
    wave_sync();
    for (int l = a.L - 1; l >= 0; --l) {
      const LayerP p = layer_params(lds, a, l);
      const int Fi = p.Fi;
      const float* xl = W + bl.xl[l];
      const float* xr = W + bl.xr[l];
      const float* al = W + bl.al[l];
      const float* hin = W + bl.hin[l];
      if (relu_after(a, l)) {
        // ReLU mask: output of conv l is hin[l+1] (post-ReLU) for l < L-1, else ylast
        const float* post = (l + 1 < a.L) ? W + bl.hin[l + 1] : W + bl.ylast;
        for (int i = lane; i < n * H; i += 64) dy[i] = post[i] > 0.f ? dy[i] : 0.f;
        wave_sync();
      }
      const int o_Wl = p.off, o_bl = o_Wl + H * Fi, o_Wr = o_bl + H, o_br = o_Wr + H * Fi;
      const int o_att = o_br + H, o_bias = o_att + H;
      for (int c = lane; c < H; c += 64) {
        float s = 0.f;
        for (int v = 0; v < n; ++v) s += dy[v * H + c];
        acc[o_bias + c] += s;
      }
      clk.mark(2);
      // d alpha_q = (dy[i] / deg_i) . x_l[j]
      for (int q = lane; q < m; q += 64) {
        const int j = T.src[q], i = T.dst[q];
        const float* gi_ = dy + i * H;
        const float* xj = xl + j * H;
        float s = 0.f;
#pragma unroll 4
        for (int c = 0; c < H; ++c) s = fmaf(gi_[c], xj[c], s);
        da[q] = s / T.deg[i];
      }
      wave_sync();
      clk.mark(3);
      // softmax backward: de_q = alpha_q (da_q - sum_{q' -> i} alpha_q' da_q')
      for (int v = lane; v < n; v += 64) {
        float sad = 0.f;
        for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) sad = fmaf(al[T.imsg[q]], da[T.imsg[q]], sad);
        for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) {
          const int mi = T.imsg[q];
          da[mi] = al[mi] * (da[mi] - sad);
        }
      }
      wave_sync();
      clk.mark(4);
      // d att_c = sum_q de_q * lrelu(z_qc)
      for (int c = lane; c < H; c += 64) {
        float s = 0.f;
        for (int q = 0; q < m; ++q) {
          float z = xl[T.src[q] * H + c] + xr[T.dst[q] * H + c];
          z = z > 0.f ? z : kNegSlope * z;
          s = fmaf(da[q], z, s);
        }
        acc[o_att + c] += s;
      }
      clk.mark(5);
      // dz_qc = de_q att_c lrelu'(z_qc);  dxl[j] = sum_{q: src=j} alpha_q dy[dst]/deg + dz;  dxr[i] = sum_{q: dst=i} dz
      for (int idx = lane; idx < n * H; idx += 64) {
        const int v = fdiv(idx, invH), c = idx - v * H;
        const float attc = p.att[c];
        const float xlv = xl[v * H + c], xrv = xr[v * H + c];
        float sl = 0.f, sr = 0.f;
        for (int q = T.optr[v]; q < T.optr[v + 1]; ++q) {
          const int mi = T.omsg[q];
          const int i = T.dst[mi];
          const float z = xlv + xr[i * H + c];
          sl = fmaf(al[mi], dy[i * H + c] / T.deg[i], sl);
          sl = fmaf(da[mi] * attc, z > 0.f ? 1.f : kNegSlope, sl);
        }
        for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) {
          const int mi = T.imsg[q];
          const float z = xl[T.src[mi] * H + c] + xrv;
          sr = fmaf(da[mi] * attc, z > 0.f ? 1.f : kNegSlope, sr);
        }
        dxl[idx] = sl;
        dxr[idx] = sr;
      }
      wave_sync();
      clk.mark(6);
      const float invFi = 1.f / (float)Fi;
      for (int idx = lane; idx < H * Fi; idx += 64) {
        const int c = fdiv(idx, invFi), k = idx - c * Fi;
        float sl = 0.f, sr = 0.f;
        for (int v = 0; v < n; ++v) {
          const float h = hin[v * Fi + k];
          sl = fmaf(dxl[v * H + c], h, sl);
          sr = fmaf(dxr[v * H + c], h, sr);
        }
        acc[o_Wl + idx] += sl;
        acc[o_Wr + idx] += sr;
      }
      clk.mark(7);
      for (int c = lane; c < H; c += 64) {
        float sl = 0.f, sr = 0.f;
        for (int v = 0; v < n; ++v) { sl += dxl[v * H + c]; sr += dxr[v * H + c]; }
        acc[o_bl + c] += sl;
        acc[o_br + c] += sr;
      }
      clk.mark(8);
      if (l > 0) {
        wave_sync();
        for (int idx = lane; idx < n * Fi; idx += 64) {
          const int v = fdiv(idx, invFi), k = idx - v * Fi;
          const float* gl = dxl + v * H;
          const float* gr = dxr + v * H;
          float s = 0.f;
#pragma unroll 2
          for (int c = 0; c < H; ++c) {
            s = fmaf(gl[c], p.Wl[c * Fi + k], s);
            s = fmaf(gr[c], p.Wr[c * Fi + k], s);
          }
          dy[idx] = s;
        }
      }
      wave_sync();
      clk.mark(9);
    }
  }
  clk.flush(a.prof, lane);
  __syncthreads();
  // reduce the waves' accumulators into this workgroup's partial row
  const float* acc0 = lds + ((a.n_params + 3) & ~3) + bl.acc;
  for (int i = tid; i < a.n_params; i += blockDim.x) {
    float s = 0.f;
    for (int w = 0; w < a.waves; ++w) s += acc0[(long)w * bl.per_wave + i];
    a.partials[(long)blockIdx.x * a.n_params + i] = s;
  }
}

// out[c] = sum_r partials[r, c]: 8 row-groups x 32 columns per block, LDS tree over the groups.
__global__ __launch_bounds__(256) void column_sum_kernel(const float* __restrict__ partials, float* __restrict__ out,
                                                         int rows, int cols) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols)
    for (int r = rg; r < rows; r += 8) s += partials[(long)r * cols + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < cols) {
    float t = 0.f;
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    out[c] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
// channel-lane fast path (gnn_cl.hip); ClArgs is GnnArgs + the number of distinct parameter blocks
struct ClArgsMirror {
  const float* params;
  const float* x;
  const int32_t *topo, *in_src, *in_dst, *in_ptr, *out_q, *out_ptr, *out_dst;
  const float* deg;
  const int32_t *nnodes, *nmsgs;
  float* emb;
  const float* demb;
  float* partials;
  int B, P, Fin, H, L, M, NM, n_params, n_blocks, waves;
  int layer_of[kGnnMaxLayers];
  unsigned long long* prof;
  const void* s_dst;
  const void* s_src;
  int MP;
  void* blob;
};
bool gnn_cl_supported(int Fin, int H, int L, int n_blocks);
bool gnn_nl_supported(int Fin, int H, int NP, int L);
void gnn_nl_forward(const float* params, int n_blocks, const float* x, const int32_t* topo, const int32_t* in_src,
                    const int32_t* in_ptr, const float* deg, const int32_t* nnodes, float* emb, int B, int P, int Fin,
                    int H, int L, int M, int NP, const int* layer_of, uintptr_t stream, int cus);
void gnn_cl_forward(const void* args, uintptr_t stream, int cus);
int gnn_cl_backward(const void* args, uintptr_t stream, int cus, int max_rows);
bool gnn_mf_supported(int Fin, int H, int NM, int L, int n_blocks, const int* layer_of);
void gnn_mf_forward(const void* args, uintptr_t stream, int cus);
int gnn_mf_backward(const void* args, uintptr_t stream, int cus, int max_rows);
int gnn_mf_saved_bytes(const void* args);

static unsigned long long* g_gnn_prof = nullptr;  // device buffer of 12 counters, or null
void gnn_set_profile(uintptr_t p) { g_gnn_prof = reinterpret_cast<unsigned long long*>(p); }
static ClArgsMirror to_cl(const GnnArgs& a, py::dict t) {
  ClArgsMirror c{};
  c.params = a.params; c.x = a.x; c.topo = a.topo;
  c.in_src = ptr<const int32_t>(t["in_src"].cast<uintptr_t>());
  c.in_dst = ptr<const int32_t>(t["in_dst"].cast<uintptr_t>());
  c.out_q = ptr<const int32_t>(t["out_q"].cast<uintptr_t>());
  c.out_dst = ptr<const int32_t>(t["out_dst"].cast<uintptr_t>());
  c.in_ptr = a.in_ptr; c.out_ptr = a.out_ptr; c.deg = a.deg; c.nnodes = a.nnodes;
  c.nmsgs = a.nmsgs; c.emb = a.emb; c.demb = a.demb; c.partials = a.partials;
  c.B = a.B; c.P = a.P; c.Fin = a.Fin; c.H = a.H; c.L = a.L; c.M = a.M; c.NM = a.NM; c.n_params = a.n_params;
  int maxb = 0;
  for (int i = 0; i < a.L; ++i) { c.layer_of[i] = a.layer_of[i]; maxb = a.layer_of[i] > maxb ? a.layer_of[i] : maxb; }
  c.n_blocks = maxb + 1;
  c.waves = 4;
  c.prof = g_gnn_prof;
  if (t.contains("s_dst")) {
    c.s_dst = reinterpret_cast<const void*>(t["s_dst"].cast<uintptr_t>());
    c.s_src = reinterpret_cast<const void*>(t["s_src"].cast<uintptr_t>());
    c.MP = t["MP"].cast<int>();
  }
  return c;
}

// Path bits: bit0 channel-lane forward, bit1 channel-lane backward, bit2 node-lane forward (forced),
// bit3 automatic node-lane forward for large graphs, bit4 MFMA forward, bit5 MFMA backward.
// Default: MFMA kernels (gnn_mf.hip) where they apply, else channel-lane, else generic.
// 25.6k Abilene graphs on MI355X: channel-lane forward 143 us / backward 924 us (generic 200 / 945).
// GSC_GNN_GENERIC=1 selects the generic kernels, GSC_GNN_CL=1 the channel-lane ones (no MFMA),
// GSC_GNN_CL_FWD_ONLY=1 only the channel-lane forward.
static int g_gnn_path = -1;
static int gnn_path() {
  if (g_gnn_path < 0)
    g_gnn_path = getenv("GSC_GNN_GENERIC") ? 0
                 : getenv("GSC_GNN_CL_FWD_ONLY") ? 1
                 : getenv("GSC_GNN_CL") ? (3 | 8)
                 : (3 | 8 | 16 | 32);
  return g_gnn_path;
}
void gnn_set_path(int bits) { g_gnn_path = bits & 63; }
static int max_block(const GnnArgs& a) {
  int maxb = 0;
  for (int i = 0; i < a.L; ++i) maxb = a.layer_of[i] > maxb ? a.layer_of[i] : maxb;
  return maxb;
}
static bool use_cl(const GnnArgs& a, bool backward = false) {
  const bool off = !(gnn_path() & (backward ? 2 : 1));
  return !off && gnn_cl_supported(a.Fin, a.H, a.L, max_block(a) + 1);
}
static bool use_mf(const GnnArgs& a, py::dict t, bool backward = false) {
  const bool off = !(gnn_path() & (backward ? 32 : 16));
  const bool uniq = t.contains("uniq") && t["uniq"].cast<bool>() && t.contains("s_dst");
  return !off && uniq && gnn_mf_supported(a.Fin, a.H, a.NM, a.L, max_block(a) + 1, a.layer_of);
}
static GnnArgs make_args(py::dict t, uintptr_t params, uintptr_t x, uintptr_t topo, int B, int P, int Fin, int H,
                         std::vector<int> layer_of) {
  GnnArgs a{};
  a.params = ptr<const float>(params);
  a.x = ptr<const float>(x);
  a.topo = ptr<const int32_t>(topo);
  a.src = ptr<const int32_t>(t["src"].cast<uintptr_t>());
  a.dst = ptr<const int32_t>(t["dst"].cast<uintptr_t>());
  a.in_ptr = ptr<const int32_t>(t["in_ptr"].cast<uintptr_t>());
  a.in_msg = ptr<const int32_t>(t["in_msg"].cast<uintptr_t>());
  a.out_ptr = ptr<const int32_t>(t["out_ptr"].cast<uintptr_t>());
  a.out_msg = ptr<const int32_t>(t["out_msg"].cast<uintptr_t>());
  a.deg = ptr<const float>(t["deg"].cast<uintptr_t>());
  a.nnodes = ptr<const int32_t>(t["nnodes"].cast<uintptr_t>());
  a.nmsgs = ptr<const int32_t>(t["nmsgs"].cast<uintptr_t>());
  a.M = t["M"].cast<int>();
  a.NM = t["NM"].cast<int>();
  a.B = B;
  a.P = P;
  a.Fin = Fin;
  a.H = H;
  GSC_CHECK((int)layer_of.size() <= kGnnMaxLayers && !layer_of.empty(), "1..16 conv applications");
  GSC_CHECK(H < 256 && Fin < 256 && a.NM * (H > Fin ? H : Fin) < 65536, "GNN dims out of range");
  a.L = (int)layer_of.size();
  int maxb = 0;
  for (int i = 0; i < a.L; ++i) {
    a.layer_of[i] = layer_of[i];
    maxb = layer_of[i] > maxb ? layer_of[i] : maxb;
  }
  a.n_params = block_offset(maxb, Fin, H) + block_size(maxb == 0 ? Fin : H, H);
  return a;
}

// CUs the launching stream may use: the device's count, or the budget of a CU-masked learner
// stream (gnn_set_cu_budget) so persistent grids are sized to one full round on that partition.
static int g_cu_budget = 0;
void gnn_set_cu_budget(int n) { g_cu_budget = n > 0 ? n : 0; }
static int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    GSC_HIP_CHECK(hipGetDevice(&dev));
    GSC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return g_cu_budget > 0 && g_cu_budget < cus ? g_cu_budget : cus;
}

static void set_lds(const void* fn, size_t lds) {
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
}

void gnn_forward(py::dict tables, uintptr_t params, uintptr_t x, uintptr_t topo, uintptr_t emb, int B, int P, int Fin,
                 int H, std::vector<int> layer_of, uintptr_t stream, uintptr_t blob) {
  GnnArgs a = make_args(tables, params, x, topo, B, P, Fin, H, layer_of);
  a.emb = ptr<float>(emb);
  // node-lane forward: forced by path bit 2, and chosen automatically for graphs with >= 32 node
  // slots (50-node synthetic: 833 us vs 1737 us channel-lane per 25.6k graphs; Abilene: a tie)
  const bool nl_auto = g_gnn_path < 0 || (g_gnn_path & 8);
  if (((gnn_path() & 4) || (nl_auto && a.NM >= 32 && (gnn_path() & 1))) && gnn_nl_supported(Fin, H, a.NM, a.L)) {
    int maxb = 0;
    for (int i = 0; i < a.L; ++i) maxb = a.layer_of[i] > maxb ? a.layer_of[i] : maxb;
    gnn_nl_forward(a.params, maxb + 1, a.x, a.topo, ptr<const int32_t>(tables["in_src"].cast<uintptr_t>()), a.in_ptr,
                   a.deg, a.nnodes, a.emb, B, P, Fin, H, a.L, a.M, a.NM, a.layer_of, stream, num_cus());
    return;
  }
  if (use_mf(a, tables)) {
    ClArgsMirror c = to_cl(a, tables);
    // the saved state is only consumed by the MFMA backward
    c.blob = blob && use_mf(a, tables, true) ? reinterpret_cast<void*>(blob) : nullptr;
    gnn_mf_forward(&c, stream, num_cus());
    return;
  }
  if (use_cl(a)) {
    const ClArgsMirror c = to_cl(a, tables);
    gnn_cl_forward(&c, stream, num_cus());
    return;
  }
  a.waves = 4;
  while (a.waves > 1 && sizeof(float) * (((a.n_params + 3) & ~3) + (size_t)a.waves * fwd_per_wave(a)) > 80 * 1024)
    a.waves--;
  const size_t lds = sizeof(float) * (((a.n_params + 3) & ~3) + (size_t)a.waves * fwd_per_wave(a));
  GSC_CHECK(lds <= 160 * 1024, "GNN forward working set exceeds LDS");
  const int blocks_needed = (B + a.waves - 1) / a.waves;
  int grid = blocks_needed < num_cus() * 8 ? blocks_needed : num_cus() * 8;
  if (grid < 1) grid = 1;
  set_lds((const void*)gnn_fwd_kernel, lds);
  hipLaunchKernelGGL(gnn_fwd_kernel, dim3(grid), dim3(64 * a.waves), lds, stream_of(stream), a);
  check_launch();
}

void gnn_backward(py::dict tables, uintptr_t params, uintptr_t x, uintptr_t topo, uintptr_t demb, uintptr_t partials,
                  int max_rows, uintptr_t grad_out, int B, int P, int Fin, int H, std::vector<int> layer_of,
                  uintptr_t stream, uintptr_t blob) {
  GnnArgs a = make_args(tables, params, x, topo, B, P, Fin, H, layer_of);
  a.demb = ptr<const float>(demb);
  a.partials = ptr<float>(partials);
  if (use_mf(a, tables, true) || use_cl(a, true)) {
    ClArgsMirror c = to_cl(a, tables);
    c.blob = reinterpret_cast<void*>(blob);
    const int rows = use_mf(a, tables, true) ? gnn_mf_backward(&c, stream, num_cus(), max_rows)
                                     : gnn_cl_backward(&c, stream, num_cus(), max_rows);
    hipLaunchKernelGGL(column_sum_kernel, dim3((a.n_params + 31) / 32), dim3(256), 0, stream_of(stream),
                       (const float*)a.partials, ptr<float>(grad_out), rows, a.n_params);
    check_launch();
    return;
  }
  BwdLayout bl{};
  a.waves = 4;
  for (;;) {
    bl = bwd_layout(a);
    const size_t lds = sizeof(float) * (((a.n_params + 3) & ~3) + (size_t)a.waves * bl.per_wave);
    if (lds <= 80 * 1024 || a.waves == 1) break;
    a.waves--;
  }
  const size_t lds = sizeof(float) * (((a.n_params + 3) & ~3) + (size_t)a.waves * bl.per_wave);
  GSC_CHECK(lds <= 160 * 1024, "GNN backward working set exceeds LDS (graph too large for the fused kernel)");
  const int per_cu = lds <= 40 * 1024 ? 4 : (lds <= 53 * 1024 ? 3 : (lds <= 80 * 1024 ? 2 : 1));
  const int blocks_needed = (B + a.waves - 1) / a.waves;
  int grid = blocks_needed < num_cus() * per_cu ? blocks_needed : num_cus() * per_cu;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  a.prof = g_gnn_prof;
  if (a.prof) {
    set_lds((const void*)gnn_bwd_kernel<true>, lds);
    hipLaunchKernelGGL(gnn_bwd_kernel<true>, dim3(grid), dim3(64 * a.waves), lds, stream_of(stream), a, bl);
  } else {
    set_lds((const void*)gnn_bwd_kernel<false>, lds);
    hipLaunchKernelGGL(gnn_bwd_kernel<false>, dim3(grid), dim3(64 * a.waves), lds, stream_of(stream), a, bl);
  }
  check_launch();
  const int cols = a.n_params;
  hipLaunchKernelGGL(column_sum_kernel, dim3((cols + 31) / 32), dim3(256), 0, stream_of(stream),
                     (const float*)a.partials, ptr<float>(grad_out), grid, cols);
  check_launch();
}

// Whether the fused kernels' per-graph working sets fit LDS (one wave per block) for these sizes;
// larger graphs (e.g. 200-node topologies) run the PyTorch reference path instead.
bool gnn_fused_fits(int M, int NM, int P, int Fin, int H, std::vector<int> layer_of) {
  GnnArgs a{};
  a.M = M; a.NM = NM; a.P = P; a.Fin = Fin; a.H = H; a.L = (int)layer_of.size(); a.waves = 1;
  if (a.L < 1 || a.L > kGnnMaxLayers) return false;
  int maxb = 0;
  for (int i = 0; i < a.L; ++i) { a.layer_of[i] = layer_of[i]; maxb = layer_of[i] > maxb ? layer_of[i] : maxb; }
  a.n_params = block_offset(maxb, Fin, H) + block_size(maxb == 0 ? Fin : H, H);
  const size_t pbytes = sizeof(float) * ((a.n_params + 3) & ~3);
  const size_t fwd = pbytes + sizeof(float) * fwd_per_wave(a);
  const size_t bwd = pbytes + sizeof(float) * bwd_layout(a).per_wave;
  return fwd <= 160 * 1024 && bwd <= 160 * 1024;
}

// Bytes per graph the grad-requiring forward saves for the MFMA backward (0: that path does not apply).
int gnn_saved_bytes(py::dict tables, int P, int Fin, int H, std::vector<int> layer_of) {
  GnnArgs a = make_args(tables, 0, 0, 0, 1, P, Fin, H, layer_of);
  if (!use_mf(a, tables) || !use_mf(a, tables, true)) return 0;
  const ClArgsMirror c = to_cl(a, tables);
  return gnn_mf_saved_bytes(&c);
}

int gnn_num_params(int Fin, int H, int max_block) { return block_offset(max_block, Fin, H) + block_size(max_block == 0 ? Fin : H, H); }

void register_gnn(py::module_& m) {
  m.def("gnn_forward", &gnn_forward, py::arg("tables"), py::arg("params"), py::arg("x"), py::arg("topo"), py::arg("emb"),
        py::arg("B"), py::arg("P"), py::arg("Fin"), py::arg("H"), py::arg("layer_of"), py::arg("stream"),
        py::arg("blob") = 0);
  m.def("gnn_backward", &gnn_backward, py::arg("tables"), py::arg("params"), py::arg("x"), py::arg("topo"),
        py::arg("demb"), py::arg("partials"), py::arg("max_rows"), py::arg("grad_out"), py::arg("B"), py::arg("P"),
        py::arg("Fin"), py::arg("H"), py::arg("layer_of"), py::arg("stream"), py::arg("blob") = 0);
  m.def("gnn_saved_bytes", &gnn_saved_bytes, "per-graph bytes of the forward state saved for the MFMA backward");
  m.def("gnn_num_params", &gnn_num_params);
  m.def("gnn_fused_fits", &gnn_fused_fits);
  m.def("gnn_set_cu_budget", &gnn_set_cu_budget, "CUs available to GNN launches (0 = whole device)");
  m.def("gnn_set_profile", &gnn_set_profile, "device int64[12] phase-cycle counters for the generic backward (0 = off)");
  m.def("gnn_set_path", &gnn_set_path, "bit0/1: channel-lane fwd/bwd, bit2: node-lane fwd, bit3: auto node-lane, bit4/5: MFMA fwd/bwd");
  m.def("gnn_get_path", &gnn_path);
}

}  // namespace gsc
