// Fused GATv2 embedder for large graphs (65 .. 256 nodes: the 200-node synthetic topologies of BASELINE
// config 5), one graph per 512-thread workgroup with every conv of the graph resident in LDS.
// Reference semantics: PyG GATv2Conv (aggr='mean', self loops, slope 0.2) as in src/rlsp/agents/models.py:10-53
// (GNNEmbedder.forward :37-53), here gsc_amd/models/gnn.py::gatv2_dense_reference.
//
// Why a separate family: the per-conv layer-wise kernels (gnn_lw.hip) stream every conv's x_l / x_r / output /
// alpha through HBM (~92 KB per graph and conv); at B = 25,600 graphs that is ~2.4 GB per conv and the kernels
// sit at ~4 TB/s -- HBM-bound, not compute-bound (a 200-node conv is ~0.5 MFLOP).  Here only the inputs
// (x: P x F_in floats) and the embedding (H floats) touch HBM; everything in between lives in LDS:
//
//   node linears  [x_l | x_r] = h W^T + b   v_mfma_f32_32x32x16_bf16, one 32-node row tile per wave, from the
//                                          conv-input image S (bf16 [node][k]) into fp32 rows XL / XR
//   attention     lane pair (2i, 2i+1) = target node i, 12 channels each (the score's channel sum is one DPP
//                 swap); online segment softmax over the CSR in-messages, mean aggregation, bias, ReLU
//   output        bf16 rows into the next conv's S image; the last conv's rows pooled into emb
//
// The backward recomputes the forward in LDS (nothing saved in HBM; convs 0 .. L-2 keep their bf16 outputs
// as the later convs' S images) and runs per conv, last to first:
//   1  x_l, x_r again (MFMA) + the transposed input image HT [k][node] (+ a ones row: bias gradients)
//   2  per target i: scores, softmax, d alpha = dY_i . x_l[j] / deg_i, d score, d x_r[i]  (VALU)
//   3  per source j through the source-sorted CSR: d x_l[j], d att  (VALU, no atomics)
//   4  d x_l, d x_r as transposed bf16 images DT [c][node] and row images DN [node][c]
//   5  MFMA: dW_l|db_l += DT_l HT^T, dW_r|db_r += DT_r HT^T (accumulated in registers over all the graphs
//      of the workgroup), dX = DN_l W_l + DN_r W_r for the conv below
//   6  dY of the conv below = dX * (h > 0)
// Per-workgroup gradient rows are summed by gnn.hip's column sum (fixed order: bitwise reproducible).
//
// The sparse parts (scores / softmax / aggregation over ~5 messages per node, 2.5 % adjacency density at 200
// nodes) stay on the VALU: a block-dense MFMA aggregation over the 7 x 7 tiles of 32 nodes would do ~50x the
// useful FLOPs (3x the VALU time at the 16:1 MFMA:VALU rate) and need a 100 KB dense alpha image per graph.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <vector>

#include "../common.h"
#include "gnn_mf.h"

namespace py = pybind11;

namespace gsc {

constexpr int kLgThreads = 512;  // 8 waves: 256 lane pairs = up to 256 nodes, 8 MFMA row tiles
constexpr int kLgMaxNodes = 256;
constexpr int kLgRows = kLgThreads / 16;  // 16-lane DPP rows of the workgroup (partial sums of the reductions)
constexpr float kLgSlope = 0.2f;
constexpr int kLgUf = 2;
constexpr int kLgUb = 2;  // ... in the backward's row-reading loops  // messages per chunk in the forward attention loop (registers: 4 waves / SIMD)

struct LgLayout {
  int P, P32, PK, RS, TS, L, nslots, xs;
  int frag, vec, ord, iptr, deg, isrc, optr, oq, odst, sc, ds, zb, slot[kClMaxLayers], R, xl, xr, dy, dtl, dtr, dnl, dnr, ht,
      red, acc0, total;
};

// thread id through an opaque asm: the LDS addresses derived from it are recomputed at their use instead of
// being hoisted out of the graph / conv loops (dozens of loop-invariant per-channel addresses otherwise stay live
// and spill)
__device__ __forceinline__ int lg_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

// Optional per-phase cycle counters (GSC_LG_PROF=1: the PROF kernel variants): thread 0 of each workgroup adds the
// s_memtime deltas between the workgroup's barriers into lg_prof[phase] (global atomics at the end)
struct LgClock {
  unsigned long long last, ph[16];
};
#define LG_MARK(PROF, clk, k)                                  \
  do {                                                         \
    if (PROF && threadIdx.x == 0) {                            \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      clk.ph[k] += t_ - clk.last;                              \
      clk.last = t_;                                           \
    }                                                          \
  } while (0)
static unsigned long long* g_lg_prof = nullptr;

// sum of v over the 8 lanes of this lane's parity in its 16-lane row (node lanes holding the same channels),
// complete in lanes 14 (even) and 15 (odd): three DPP row shifts, no LDS
__device__ __forceinline__ float lg_row_parity_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));  // row_shr:2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false));  // row_shr:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false));  // row_shr:8
  return v;
}

// lane value of the pair partner (lanes 2i <-> 2i+1): DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ float lg_pair(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

template <int HC>
__device__ __forceinline__ void lg_load_f(float (&v)[HC], const float* src) {
#pragma unroll
  for (int u = 0; u < HC / 4; ++u) {
    const float4 f = reinterpret_cast<const float4*>(src)[u];
    v[4 * u] = f.x;
    v[4 * u + 1] = f.y;
    v[4 * u + 2] = f.z;
    v[4 * u + 3] = f.w;
  }
}
template <int HC>
__device__ __forceinline__ void lg_store_bf16(__bf16* dst, const float (&v)[HC]) {  // HC / 4 8-byte stores
#pragma unroll
  for (int u = 0; u < HC / 4; ++u) {
    bf16x4 b;
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[4 * u + e];
    reinterpret_cast<bf16x4*>(dst)[u] = b;
  }
}
template <int HC>
__device__ __forceinline__ void lg_load_bf16(float (&v)[HC], const __bf16* src) {
#pragma unroll
  for (int u = 0; u < HC / 4; ++u) {
    const bf16x4 b = reinterpret_cast<const bf16x4*>(src)[u];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * u + e] = (float)b[e];
  }
}

// Weight fragments of the node linears (set 2b: block b, B operand of h W^T) and of the input gradient (set
// 2: block 1 transposed, B operand of dX W), lane-linear in LDS: [set][Wl k-step 0, 1, Wr k-step 0, 1][lane]
__device__ __forceinline__ void lg_stage_frags(const ClArgs& a, bf16x8* img, int nsets) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int f = wave; f < nsets; f += kLgThreads / 64) {
    MfW w;
    mf_load_w(w, a, a.params, f == 0 ? 0 : 1, f == 2, lane);
    img[(f * 4 + 0) * 64 + lane] = w.l[0];
    img[(f * 4 + 1) * 64 + lane] = w.l[1];
    img[(f * 4 + 2) * 64 + lane] = w.r[0];
    img[(f * 4 + 3) * 64 + lane] = w.r[1];
  }
}

// X_l, X_r = S W^T + b on the matrix cores, computed transposed (X^T = W S^T: the weight fragments as the A
// operand, the S rows as B) so each lane ends with 16 channels of one node -- four runs of 4 consecutive channels
// stored as 16-byte rows (8 ds_write_b128 per node instead of 32 ds_write_b32) -- and can form the score's linear
// part u = att . x_l, v = att . x_r itself (its 16 channels + the lane 32 apart): stored in the padding channel
// HV - 1 of each row (H < HV), so the attention's |z| sum and the linear part share one row read.
// Rows < P, channels < HV; wave w takes 32-node tiles w, w + 8.
template <int HV>
__device__ __forceinline__ void lg_linear(const bf16x8* frag, int set, bool k2, const float* vec, const __bf16* S,
                                          float* XL, float* XR, const LgLayout& m) {
  const int tid = lg_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), r = lane & 31, hh = lane >> 5;
  const bf16x8* fs = frag + set * 4 * 64;
  for (int t = wave; 32 * t < m.P32; t += kLgThreads / 64) {
    f32x16 al, ar;
    float at[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // accumulator rows 4g .. 4g+3 = channels 8g + 4hh + (0..3)
      const float4 bl = *reinterpret_cast<const float4*>(vec + 8 * g + 4 * hh);
      const float4 br = *reinterpret_cast<const float4*>(vec + 32 + 8 * g + 4 * hh);
      const float4 aa = *reinterpret_cast<const float4*>(vec + 64 + 8 * g + 4 * hh);
      al[4 * g] = bl.x; al[4 * g + 1] = bl.y; al[4 * g + 2] = bl.z; al[4 * g + 3] = bl.w;
      ar[4 * g] = br.x; ar[4 * g + 1] = br.y; ar[4 * g + 2] = br.z; ar[4 * g + 3] = br.w;
      at[4 * g] = aa.x; at[4 * g + 1] = aa.y; at[4 * g + 2] = aa.z; at[4 * g + 3] = aa.w;
    }
    const int node = 32 * t + r;
    const __bf16* row = S + node * kMfRS + 8 * hh;
    const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(row);
    al = mf_mma(fs[0 * 64 + lane], b0, al);
    ar = mf_mma(fs[2 * 64 + lane], b0, ar);
    if (k2) {
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(row + 16);
      al = mf_mma(fs[1 * 64 + lane], b1, al);
      ar = mf_mma(fs[3 * 64 + lane], b1, ar);
    }
    float u = 0.f, v = 0.f;  // att is zero past H: the padding channels add nothing
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      u = fmaf(at[i], al[i], u);
      v = fmaf(at[i], ar[i], v);
    }
    u += __shfl_xor(u, 32);
    v += __shfl_xor(v, 32);
    constexpr int gs = HV / 8 - 1;  // channel HV - 1 = row 4 gs + 3 of lane half 1
    if (hh == 1) {
      al[4 * gs + 3] = u;
      ar[4 * gs + 3] = v;
    }
    if (node < m.P) {
      float* xl = XL + node * m.RS + 4 * hh;
      float* xr = XR + node * m.RS + 4 * hh;
#pragma unroll
      for (int g = 0; g < HV / 8; ++g) {
        *reinterpret_cast<float4*>(xl + 8 * g) = float4{al[4 * g], al[4 * g + 1], al[4 * g + 2], al[4 * g + 3]};
        *reinterpret_cast<float4*>(xr + 8 * g) = float4{ar[4 * g], ar[4 * g + 1], ar[4 * g + 2], ar[4 * g + 3]};
      }
    }
  }
}

// Forward attention of target node i (lane pair, channels c0 .. c0 + HC): PyG segment softmax (online, one
// rescale per chunk) and mean aggregation; returns the conv output half-row (bias, optional ReLU; zero for i >= n).
// Messages go U at a time: the U source ids, then the U rows are loaded before any of them is used (clamped to
// the segment's last message), so one LDS round trip serves U messages.
template <int HC, int U>
__device__ __forceinline__ void lg_attend(float (&y)[HC], int i, int n, int c0, const float* vec, bool relu,
                                          const float* XL, const float* XR, const int32_t* iptr,
                                          const uint16_t* isrc, const float* deg, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) y[k] = 0.f;
  if (i >= n) return;
  // score = att . LeakyReLU(z) = 0.6 (u_j + v_i) + 0.4 att . |z|: one FMA per channel with the |z| source
  // modifier; the half holding channel HV - 1 (u + v) adds the linear part
  const bool hi = c0 != 0;
  float xr[HC], a4[HC], acc[HC];
  lg_load_f<HC>(xr, XR + i * m.RS + c0);
  lg_load_f<HC>(a4, vec + 64 + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    a4[k] *= 0.5f * (1.f - kLgSlope);
    acc[k] = 0.f;
  }
  const float lin = hi ? 0.5f * (1.f + kLgSlope) : 0.f;
  const int q0 = iptr[i], q1 = iptr[i + 1];
  float mx = -__builtin_inff(), den = 0.f;
  for (int q = q0; q < q1; q += U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = isrc[min(q + u, q1 - 1)];
    float xj[U][HC];
#pragma unroll
    for (int u = 0; u < U; ++u) lg_load_f<HC>(xj[u], XL + j[u] * m.RS + c0);
    float sc[U];
    float cm = -__builtin_inff();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float z[HC];
#pragma unroll
      for (int k = 0; k < HC; ++k) z[k] = xj[u][k] + xr[k];
      float v = lin * z[HC - 1];
#pragma unroll
      for (int k = 0; k < HC; ++k) v = fmaf(a4[k], fabsf(z[k]), v);
      v += lg_pair(v);
      sc[u] = q + u < q1 ? v : -__builtin_inff();
      cm = fmaxf(cm, sc[u]);
    }
    if (cm > mx) {
      const float rs = __expf(mx - cm);  // 0 for the first chunk
      den *= rs;
#pragma unroll
      for (int k = 0; k < HC; ++k) acc[k] *= rs;
      mx = cm;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float e = __expf(sc[u] - mx);  // 0 past the segment
      den += e;
#pragma unroll
      for (int k = 0; k < HC; ++k) acc[k] = fmaf(e, xj[u][k], acc[k]);
    }
  }
  const float scl = 1.f / ((den + 1e-16f) * deg[i]);
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    float v = fmaf(acc[k], scl, vec[96 + c0 + k]);
    y[k] = relu ? fmaxf(v, 0.f) : v;
  }
  if (hi) y[HC - 1] = 0.f;  // channel HV - 1 carried u: not an output channel
}

// Topology rows of graph type t into LDS (u16 message arrays; the backward also the source-sorted CSR)
template <bool BWD>
__device__ __forceinline__ void lg_stage_topo(const ClArgs& a, int t, char* lds, const LgLayout& m) {
  int32_t* iptr = reinterpret_cast<int32_t*>(lds + m.iptr);
  float* deg = reinterpret_cast<float*>(lds + m.deg);
  uint16_t* isrc = reinterpret_cast<uint16_t*>(lds + m.isrc);
  const int P = m.P, M = a.M;
  uint16_t* ord = reinterpret_cast<uint16_t*>(lds + m.ord);
  for (int k = threadIdx.x; k < 2 * P; k += kLgThreads) ord[k] = (uint16_t)a.deg_order[(long)t * 2 * P + k];
  for (int k = threadIdx.x; k <= P; k += kLgThreads) {
    iptr[k] = a.in_ptr[(long)t * (P + 1) + k];
    if (k < P) deg[k] = a.deg[(long)t * P + k];
    if (BWD) reinterpret_cast<int32_t*>(lds + m.optr)[k] = a.out_ptr[(long)t * (P + 1) + k];
  }
  for (int k = threadIdx.x; k < M; k += kLgThreads) {
    isrc[k] = (uint16_t)a.in_src[(long)t * M + k];
    if (BWD) {
      reinterpret_cast<uint16_t*>(lds + m.oq)[k] = (uint16_t)a.out_q[(long)t * M + k];
      reinterpret_cast<uint16_t*>(lds + m.odst)[k] = (uint16_t)a.out_dst[(long)t * M + k];
    }
  }
}

// input rows of graph b as the bf16 image (channels 0..15: F_in <= 16, zero past F_in and for rows >= P)
__device__ __forceinline__ void lg_load_x(float (&xv)[8], const ClArgs& a, long b, int i, int hf) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = 8 * hf + k;
    xv[k] = (i < a.P && c < a.Fin) ? a.x[(b * a.P + i) * a.Fin + c] : 0.f;
  }
}
__device__ __forceinline__ void lg_put_x(__bf16* S, const float (&xv)[8], int i, int hf, const LgLayout& m) {
  if (i < m.P32) {
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (__bf16)xv[k];
    *reinterpret_cast<bf16x8*>(S + i * kMfRS + 8 * hf) = v;
  }
}

__device__ __forceinline__ void lg_zero(char* p, int bytes) {
  for (int k = 16 * threadIdx.x; k < bytes; k += 16 * kLgThreads) *reinterpret_cast<float4*>(p + k) = float4{0, 0, 0, 0};
}

// ---------------------------------------------------------------------------------------------
// forward: emb[b] = mean over real nodes of the last conv's rows (a.params2 / a.emb2: unused here; two launches)
// ---------------------------------------------------------------------------------------------
template <int HV, bool PROF>
__global__ __launch_bounds__(kLgThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void gnn_lg_fwd_kernel(ClArgs a, LgLayout m, unsigned long long* prof) {
  constexpr int HC = HV / 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  bf16x8* frag = reinterpret_cast<bf16x8*>(lds + m.frag);
  float* vec = reinterpret_cast<float*>(lds + m.vec);
  __bf16* S = reinterpret_cast<__bf16*>(lds + m.slot[0]);
  float* XL = reinterpret_cast<float*>(lds + m.xl);
  float* XR = reinterpret_cast<float*>(lds + m.xr);
  float* red = reinterpret_cast<float*>(lds + m.red);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  lg_stage_frags(a, frag, 2);
  mf_stage_vec(a, vec);
  lg_zero(reinterpret_cast<char*>(S), m.P32 * kMfRS * 2);  // channels HV..31 and rows >= P stay zero
  const bool k2b = a.H > 16;
  LgClock clk{};
  if (PROF) clk.last = __builtin_amdgcn_s_memtime();
  for (long b = blockIdx.x; b < a.B; b += gridDim.x) {
    const int t = a.topo[b], n = a.nnodes[t];
    {
      const int tq = lg_tid();
      float xv[8];
      lg_load_x(xv, a, b, tq >> 1, tq & 1);
      __syncthreads();  // the previous graph is done with every LDS image
      LG_MARK(PROF, clk, 0);
      lg_stage_topo<false>(a, t, lds, m);
      lg_put_x(S, xv, tq >> 1, tq & 1, m);
      __syncthreads();
      LG_MARK(PROF, clk, 1);
    }
    const int32_t* iptr = reinterpret_cast<const int32_t*>(lds + m.iptr);
    const uint16_t* isrc = reinterpret_cast<const uint16_t*>(lds + m.isrc);
    const float* deg = reinterpret_cast<const float*>(lds + m.deg);
    for (int l = 0; l < a.L; ++l) {
      const int blk = a.layer_of[l];
      const float* vb = vec + blk * kMfVec;
      lg_linear<HV>(frag, blk, blk ? k2b : false, vb, S, XL, XR, m);
      __syncthreads();
      LG_MARK(PROF, clk, 2);
      // lane pair p = the node of in-degree rank p (similar segment lengths per wave); p >= P: idle (zero rows)
      const int tq = lg_tid(), pq = tq >> 1, cq = (tq & 1) * HC, lane = tq & 63;
      const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
      float y[HC];
      const bool last = l + 1 == a.L;
      lg_attend<HC, kLgUf>(y, iq, n, cq, vb, !last, XL, XR, iptr, isrc, deg, m);
      if (!last) {
        __syncthreads();  // S (this conv's input) was read by the node linears before the previous barrier;
                          // the barrier orders this conv's XL reads before the next node linears' XL writes
        LG_MARK(PROF, clk, 3);
        if (iq < m.P32) lg_store_bf16<HC>(S + iq * kMfRS + cq, y);
        __syncthreads();
        LG_MARK(PROF, clk, 4);
      } else {  // mean pool over the real nodes: DPP row sums, then the 32 row partials in a fixed order
#pragma unroll
        for (int k = 0; k < HC; ++k) {
          const float v = lg_row_parity_sum(y[k]);  // y is zero for i >= n
          if ((lane & 14) == 14) red[(tq >> 4) * 32 + cq + k] = v;
        }
        __syncthreads();
        if (tq < a.H) {
          float s = 0.f;
#pragma unroll 8
          for (int w = 0; w < kLgRows; ++w) s += red[w * 32 + tq];
          a.emb[b * a.H + tq] = s / (float)n;
        }
        LG_MARK(PROF, clk, 5);
      }
    }
  }
  if (PROF && threadIdx.x == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(prof + k, clk.ph[k]);
}

// ---------------------------------------------------------------------------------------------
// backward (recompute): per-workgroup gradient rows (module layout) into a.partials[blockIdx.x]
// ---------------------------------------------------------------------------------------------
// step 2: per target node i -- softmax backward and d x_r[i]; alpha / d score per message into SC / DS.  One pass
// over the source rows (U at a time): score, z signs and d alpha = dY_i . x_l[j] / deg_i together; then two
// row-free passes over the per-message scalars.
template <int HC, int U>
__device__ __forceinline__ void lg_bwd_targets(float (&dxr)[HC], float (&gbias)[HC], int i, int n, int c0, int hf,
                                               const float* vec, char* lds, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) dxr[k] = 0.f;
  if (i >= n) return;
  const float* XL = reinterpret_cast<const float*>(lds + m.xl);
  const float* XR = reinterpret_cast<const float*>(lds + m.xr);
  const float* DY = reinterpret_cast<const float*>(lds + m.dy);
  const int32_t* iptr = reinterpret_cast<const int32_t*>(lds + m.iptr);
  const uint16_t* isrc = reinterpret_cast<const uint16_t*>(lds + m.isrc);
  const float* deg = reinterpret_cast<const float*>(lds + m.deg);
  float* SC = reinterpret_cast<float*>(lds + m.sc);
  float* DS = reinterpret_cast<float*>(lds + m.ds);
  uint16_t* ZB = reinterpret_cast<uint16_t*>(lds + m.zb);
  float xr[HC], at[HC], dy[HC];
  lg_load_f<HC>(xr, XR + i * m.RS + c0);
  lg_load_f<HC>(at, vec + 64 + c0);
  lg_load_f<HC>(dy, DY + i * m.RS + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) gbias[k] += dy[k];
  const int q0 = iptr[i], q1 = iptr[i + 1];
  const float rdeg = 1.f / deg[i];
  const float lin = hf ? 0.5f * (1.f + kLgSlope) : 0.f;  // the half holding channel HV - 1 (u + v): linear part
  float mx = -__builtin_inff(), den = 0.f;
  for (int q = q0; q < q1; q += U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = isrc[min(q + u, q1 - 1)];
    float xj[U][HC];
#pragma unroll
    for (int u = 0; u < U; ++u) lg_load_f<HC>(xj[u], XL + j[u] * m.RS + c0);
    float sc[U], da[U];
    uint32_t bits[U];
    float cm = -__builtin_inff();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float z[HC];
#pragma unroll
      for (int k = 0; k < HC; ++k) z[k] = xj[u][k] + xr[k];
      float v = lin * z[HC - 1], d = 0.f;
      bits[u] = 0;
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        v = fmaf(0.5f * (1.f - kLgSlope) * at[k], fabsf(z[k]), v);
        d = fmaf(dy[k], xj[u][k], d);
        bits[u] |= (z[k] > 0.f ? 1u : 0u) << k;
      }
      v += lg_pair(v);
      d += lg_pair(d);
      sc[u] = q + u < q1 ? v : -__builtin_inff();
      da[u] = d * rdeg;
      cm = fmaxf(cm, sc[u]);
    }
    if (cm > mx) {
      den *= __expf(mx - cm);
      mx = cm;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      den += __expf(sc[u] - mx);
      if (q + u < q1) {
        if (hf == 0) {
          SC[q + u] = sc[u];
          DS[q + u] = da[u];
        }
        ZB[2 * (q + u) + hf] = (uint16_t)bits[u];
      }
    }
  }
  // alpha = softmax; c = sum alpha d alpha (row-free: the lane's own SC / DS entries, written by the pair's
  // lane 0 in this wave, read back in program order)
  const float inv = 1.f / (den + 1e-16f);
  float cs = 0.f;
  for (int q = q0; q < q1; q += 4) {
    float sv[4], dv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sv[u] = SC[min(q + u, q1 - 1)];
      dv[u] = DS[min(q + u, q1 - 1)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float al = __expf(sv[u] - mx) * inv;
      if (q + u < q1) {
        cs = fmaf(al, dv[u], cs);
        if (hf == 0) SC[q + u] = al;
      }
    }
  }
  // d score = alpha (d alpha - c);  d x_r[i] += d score * att * LeakyReLU'(z)
  for (int q = q0; q < q1; q += 4) {
    float av[4], dv[4];
    uint32_t bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qq = min(q + u, q1 - 1);
      av[u] = SC[qq];
      dv[u] = DS[qq];
      bv[u] = ZB[2 * qq + hf];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (q + u < q1) {
        const float ds = av[u] * (dv[u] - cs);
#pragma unroll
        for (int k = 0; k < HC; ++k)
          dxr[k] = fmaf(ds * at[k], __builtin_amdgcn_ubfe(bv[u], k, 1) ? 1.f : kLgSlope, dxr[k]);
        if (hf == 0) DS[q + u] = ds;
      }
    }
  }
}

// step 3: per source node j through the source-sorted CSR -- d x_l[j] and the attention-vector gradient (U
// out-messages at a time: ids, then the target rows of x_r and dY, all loaded before use)
template <int HC, int U>
__device__ __forceinline__ void lg_bwd_sources(float (&dxl)[HC], float (&gatt)[HC], int j, int n, int c0,
                                               const float* vec, char* lds, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) dxl[k] = 0.f;
  if (j >= n) return;
  const float* XL = reinterpret_cast<const float*>(lds + m.xl);
  const float* XR = reinterpret_cast<const float*>(lds + m.xr);
  const float* DY = reinterpret_cast<const float*>(lds + m.dy);
  const int32_t* optr = reinterpret_cast<const int32_t*>(lds + m.optr);
  const uint16_t* oq = reinterpret_cast<const uint16_t*>(lds + m.oq);
  const uint16_t* odst = reinterpret_cast<const uint16_t*>(lds + m.odst);
  const float* deg = reinterpret_cast<const float*>(lds + m.deg);
  const float* SC = reinterpret_cast<const float*>(lds + m.sc);
  const float* DS = reinterpret_cast<const float*>(lds + m.ds);
  float xl[HC], at[HC];
  lg_load_f<HC>(xl, XL + j * m.RS + c0);
  lg_load_f<HC>(at, vec + 64 + c0);
  const int p0 = optr[j], p1 = optr[j + 1];
  for (int p = p0; p < p1; p += U) {
    int q[U], ti[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pp = min(p + u, p1 - 1);
      q[u] = oq[pp];
      ti[u] = odst[pp];
    }
    float xr[U][HC], dy[U][HC], w[U], ds[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lg_load_f<HC>(xr[u], XR + ti[u] * m.RS + c0);
      lg_load_f<HC>(dy[u], DY + ti[u] * m.RS + c0);
      w[u] = SC[q[u]] / deg[ti[u]];
      ds[u] = DS[q[u]];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p + u < p1) {
#pragma unroll
        for (int k = 0; k < HC; ++k) {
          const float z = xl[k] + xr[u][k];
          const bool pos = z > 0.f;
          gatt[k] = fmaf(ds[u], pos ? z : kLgSlope * z, gatt[k]);
          dxl[k] = fmaf(w[u], dy[u][k], fmaf(ds[u] * at[k], pos ? 1.f : kLgSlope, dxl[k]));
        }
      }
    }
  }
}

// HT [k][node] (bf16, row stride TS) of the conv input image S: channels < Fi, a ones row at k = Fi (bias
// gradients from the same product), zero rows in between up to HV; zero columns for nodes >= P
template <int HC>
__device__ __forceinline__ void lg_put_ht(__bf16* HT, const __bf16* S, int i, int c0, int Fi, const LgLayout& m) {
  if (i >= m.PK) return;
  float v[HC];
  if (i < m.P) lg_load_bf16<HC>(v, S + i * kMfRS + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    const int c = c0 + k;
    const float e = i >= m.P ? 0.f : (c < Fi ? v[k] : (c == Fi ? 1.f : 0.f));
    HT[c * m.TS + i] = (__bf16)e;
  }
  if (Fi >= 2 * HC && c0 == HC) HT[Fi * m.TS + i] = (__bf16)(i < m.P ? 1.f : 0.f);  // ones row past the channels
}

template <int HV, bool PROF>
__global__ __launch_bounds__(kLgThreads, 1) void gnn_lg_bwd_kernel(ClArgs a, LgLayout m, unsigned long long* prof) {
  constexpr int HC = HV / 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  bf16x8* frag = reinterpret_cast<bf16x8*>(lds + m.frag);
  float* vec = reinterpret_cast<float*>(lds + m.vec);
  __bf16* HT = reinterpret_cast<__bf16*>(lds + m.ht);
  float* XL = reinterpret_cast<float*>(lds + m.xl);
  float* XR = reinterpret_cast<float*>(lds + m.xr);
  float* DY = reinterpret_cast<float*>(lds + m.dy);
  float* red = reinterpret_cast<float*>(lds + m.red);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  lg_stage_frags(a, frag, 3);
  mf_stage_vec(a, vec);
  for (int s = 0; s < m.nslots; ++s) lg_zero(lds + m.slot[s], m.P32 * kMfRS * 2);
  lg_zero(lds + m.ht, 32 * m.TS * 2);
  const bool k2b = a.H > 16;
  // gradient accumulators over all the graphs of this workgroup: per lane (attention vector, output bias; lane
  // pair = node, 12 channels) and, in waves 0..3, the augmented weight gradients [dW | db] of (block, side)
  // (block 1, convs 1 .. L-1: registers for the workgroup's whole run; block 0, conv 0 only: per graph, then
  // summed over the wave's nodes into the wave's own LDS slot -- 24 fewer live registers)
  float gatt1[HC], gbias1[HC];
#pragma unroll
  for (int k = 0; k < HC; ++k) gatt1[k] = gbias1[k] = 0.f;
  // block 0's [att | bias][32] sums over the workgroup's graphs (thread c owns entry c of each)
  if (threadIdx.x < 64) reinterpret_cast<float*>(lds + m.acc0)[threadIdx.x] = 0.f;
  f32x16 accW;
  mf_zero(accW);
  const int wblk = wave >> 1, wside = wave & 1;  // waves 0..3: (block, l | r) of accW
  LgClock clk{};
  if (PROF) clk.last = __builtin_amdgcn_s_memtime();
  for (long b = blockIdx.x; b < a.B; b += gridDim.x) {
    const int t = a.topo[b], n = a.nnodes[t];
    float gatt0[HC], gbias0[HC];
#pragma unroll
    for (int k = 0; k < HC; ++k) gatt0[k] = gbias0[k] = 0.f;
    {
      const int tq = lg_tid(), iq = tq >> 1, hq = tq & 1, cq = hq * HC;
      float xv[8], dy0[HC];
      lg_load_x(xv, a, b, iq, hq);
#pragma unroll
      for (int k = 0; k < HC; ++k) dy0[k] = (iq < n && cq + k < a.H) ? a.demb[b * a.H + cq + k] / (float)n : 0.f;
      __syncthreads();  // the previous graph is done with every LDS image
      LG_MARK(PROF, clk, 0);
      lg_stage_topo<true>(a, t, lds, m);
      lg_put_x(reinterpret_cast<__bf16*>(lds + m.slot[m.xs]), xv, iq, hq, m);
      if (iq < m.P) {  // d emb / n on every real node (no ReLU after the last conv: L >= 2)
#pragma unroll
        for (int u = 0; u < HC / 4; ++u)
          reinterpret_cast<float4*>(DY + iq * m.RS + cq)[u] = float4{dy0[4 * u], dy0[4 * u + 1], dy0[4 * u + 2], dy0[4 * u + 3]};
      }
      __syncthreads();
      LG_MARK(PROF, clk, 1);
    }
    const int32_t* iptr = reinterpret_cast<const int32_t*>(lds + m.iptr);
    const uint16_t* isrc = reinterpret_cast<const uint16_t*>(lds + m.isrc);
    const float* deg = reinterpret_cast<const float*>(lds + m.deg);
    // ---- recompute convs 0 .. L-2; conv l's output (the input of conv l+1) is kept in slot l
    for (int l = 0; l + 1 < a.L; ++l) {
      const int blk = a.layer_of[l];
      const float* vb = vec + blk * kMfVec;
      const __bf16* Sin = reinterpret_cast<const __bf16*>(lds + m.slot[l == 0 ? m.xs : l - 1]);
      lg_linear<HV>(frag, blk, blk ? k2b : false, vb, Sin, XL, XR, m);
      __syncthreads();
      LG_MARK(PROF, clk, 2);
      const int tq = lg_tid(), pq = tq >> 1, cq = (tq & 1) * HC;
      const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
      float y[HC];
      lg_attend<HC, kLgUf>(y, iq, n, cq, vb, true, XL, XR, iptr, isrc, deg, m);
      __syncthreads();
      LG_MARK(PROF, clk, 3);
      if (iq < m.P32) lg_store_bf16<HC>(reinterpret_cast<__bf16*>(lds + m.slot[l]) + iq * kMfRS + cq, y);
      __syncthreads();
      LG_MARK(PROF, clk, 4);
    }
    // ---- backward, last conv to first
    for (int l = a.L - 1; l >= 0; --l) {
      const int blk = a.layer_of[l];
      const int Fi = blk == 0 ? a.Fin : a.H;
      const float* vb = vec + blk * kMfVec;
      __bf16* Sin = reinterpret_cast<__bf16*>(lds + m.slot[l == 0 ? m.xs : l - 1]);
      if (l == 0 && a.L >= 2) {  // the input image again (its slot held conv L-2's output meanwhile)
        const int tq = lg_tid();
        float xv[8];
        lg_load_x(xv, a, b, tq >> 1, tq & 1);
        lg_put_x(Sin, xv, tq >> 1, tq & 1, m);
        __syncthreads();
        LG_MARK(PROF, clk, 5);
      }
      // 1: x_l, x_r and HT
      lg_linear<HV>(frag, blk, blk ? k2b : false, vb, Sin, XL, XR, m);
      {
        const int tq = lg_tid();
        lg_put_ht<HC>(HT, Sin, tq >> 1, (tq & 1) * HC, Fi, m);
      }
      __syncthreads();
      LG_MARK(PROF, clk, 6);
      // 2 + 3
      // lane pair p: step 2's target = the node of in-degree rank p, step 3's source = the node of out-degree rank p
      float dxr[HC], dxl[HC];
      {
        const int tq = lg_tid(), pq = tq >> 1, hq = tq & 1;
        const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
        if (blk == 0) lg_bwd_targets<HC, kLgUb>(dxr, gbias0, iq, n, hq * HC, hq, vb, lds, m);
        else lg_bwd_targets<HC, kLgUb>(dxr, gbias1, iq, n, hq * HC, hq, vb, lds, m);
      }
      __syncthreads();
      LG_MARK(PROF, clk, 7);
      {
        const int tq = lg_tid(), pq = tq >> 1, hq = tq & 1;
        const int jq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[m.P + pq] : pq;
        if (blk == 0) lg_bwd_sources<HC, kLgUb>(dxl, gatt0, jq, n, hq * HC, vb, lds, m);
        else lg_bwd_sources<HC, kLgUb>(dxl, gatt1, jq, n, hq * HC, vb, lds, m);
      }
      __syncthreads();  // XL / XR / DY are dead: their region takes DT / DN
      LG_MARK(PROF, clk, 8);
      // 4: d x_l, d x_r images
      __bf16* DTl = reinterpret_cast<__bf16*>(lds + m.dtl);
      __bf16* DTr = reinterpret_cast<__bf16*>(lds + m.dtr);
      __bf16* DNl = reinterpret_cast<__bf16*>(lds + m.dnl);
      __bf16* DNr = reinterpret_cast<__bf16*>(lds + m.dnr);
      {
        const int tq = lg_tid(), pq = tq >> 1, hq = tq & 1, cq = hq * HC;
        const uint16_t* ord = reinterpret_cast<const uint16_t*>(lds + m.ord);
        const int iq = pq < m.P ? (int)ord[pq] : pq, jq = pq < m.P ? (int)ord[m.P + pq] : pq;
        if (pq < m.PK) {  // columns P..PK-1: zero (idle lanes hold zeros)
          __bf16* pl = DTl + cq * m.TS + jq;
          __bf16* pr = DTr + cq * m.TS + iq;
#pragma unroll
          for (int k = 0; k < HC; ++k) {
            pl[k * m.TS] = (__bf16)dxl[k];
            pr[k * m.TS] = (__bf16)dxr[k];
          }
        }
        if (l > 0 && pq < m.P32) {
          lg_store_bf16<HC>(DNl + jq * kMfRS + cq, dxl);
          lg_store_bf16<HC>(DNr + iq * kMfRS + cq, dxr);
          if (hq == 1 && HV < 32) {  // K columns HV..31 of the dX product: zero (the region held fp32 rows)
            *reinterpret_cast<bf16x8*>(DNl + jq * kMfRS + 24) = bf16x8{};
            *reinterpret_cast<bf16x8*>(DNr + iq * kMfRS + 24) = bf16x8{};
          }
        }
      }
      __syncthreads();
      LG_MARK(PROF, clk, 9);
      // 5: weight gradients (K = nodes) and the input gradient dX = dxl W_l + dxr W_r (K = channels)
      f32x16 dx;  // this wave's 32-row tile of dX (8 waves x 32 rows cover up to 256 nodes)
      const bool own_tile = 32 * wave < m.P32;
      {
        const int tq = lg_tid(), lq = tq & 63, rq = lq & 31, hq = lq >> 5;
        if (wave < 4 && wblk == blk) {
          const __bf16* DT = (wside ? DTr : DTl) + rq * m.TS + 8 * hq;
          const __bf16* HTq = HT + rq * m.TS + 8 * hq;
          for (int ks = 0; ks < m.PK / 16; ++ks) {
            const bf16x8 fa = *reinterpret_cast<const bf16x8*>(DT + 16 * ks);
            const bf16x8 fb = *reinterpret_cast<const bf16x8*>(HTq + 16 * ks);
            accW = mf_mma(fa, fb, accW);
          }
        }
        if (l > 0 && own_tile) {
          const bf16x8* fs = frag + 2 * 4 * 64;  // block 1 transposed
          mf_zero(dx);
          const __bf16* rl = DNl + (32 * wave + rq) * kMfRS + 8 * hq;
          const __bf16* rr = DNr + (32 * wave + rq) * kMfRS + 8 * hq;
          dx = mf_mma(*reinterpret_cast<const bf16x8*>(rl), fs[0 * 64 + lq], dx);
          dx = mf_mma(*reinterpret_cast<const bf16x8*>(rr), fs[2 * 64 + lq], dx);
          if (k2b) {
            dx = mf_mma(*reinterpret_cast<const bf16x8*>(rl + 16), fs[1 * 64 + lq], dx);
            dx = mf_mma(*reinterpret_cast<const bf16x8*>(rr + 16), fs[3 * 64 + lq], dx);
          }
        }
      }
      __syncthreads();  // DT / DN read: the region takes the dY rows of the conv below
      LG_MARK(PROF, clk, 10);
      // 6: dY of conv l-1 = dX * (h > 0), h = this conv's input (the ReLU output of conv l-1)
      if (l > 0) {
        const int tq = lg_tid(), lq = tq & 63, rq = lq & 31, hq = lq >> 5;
        if (own_tile && rq < HV) {
          float* dyq = DY + (32 * wave + 4 * hq) * m.RS + rq;
          const __bf16* sq = Sin + (32 * wave + 4 * hq) * kMfRS + rq;
          const int nn = m.P - 32 * wave - 4 * hq;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int ro = (e & 3) + 8 * (e >> 2);
            if (ro < nn) dyq[ro * m.RS] = (float)sq[ro * kMfRS] > 0.f ? dx[e] : 0.f;
          }
        }
        __syncthreads();
        LG_MARK(PROF, clk, 11);
      }
    }
    {  // block 0's per-graph sums: DPP row sums -> red (row partials) -> thread c adds their fixed-order sum into
       // acc0[which][c] (the last conv's barrier ordered every earlier use of red)
      const int tq = lg_tid(), cq = (tq & 1) * HC;
      float* acc0 = reinterpret_cast<float*>(lds + m.acc0);
      for (int which = 0; which < 2; ++which) {
#pragma unroll
        for (int k = 0; k < HC; ++k) {
          const float v = lg_row_parity_sum(which == 0 ? gatt0[k] : gbias0[k]);
          if ((tq & 14) == 14) red[(tq >> 4) * 32 + cq + k] = v;
        }
        __syncthreads();
        if (tq < a.H) {
          float s = 0.f;
#pragma unroll 8
          for (int w = 0; w < kLgRows; ++w) s += red[w * 32 + tq];
          acc0[which * 32 + tq] += s;
        }
        __syncthreads();
      }
    }
    LG_MARK(PROF, clk, 12);
  }
  if (PROF && threadIdx.x == 0)
    for (int k = 0; k < 13; ++k) atomicAdd(prof + 16 + k, clk.ph[k]);
  // ---- this workgroup's gradient row (module layout per block: Wl, bl, Wr, br, att, bias)
  float* row = a.partials + (long)blockIdx.x * a.n_params;
  const int H = a.H;
  const int tid = threadIdx.x, c0 = (tid & 1) * HC, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  if (wave < 4 && wblk < a.n_blocks) {
    const int Fi = wblk == 0 ? a.Fin : H, o = cl_block_offset(wblk, a.Fin, H) + wside * (H * Fi + H);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = mf_row(e, hh);
      if (c < H) {
        if (r < Fi) row[o + c * Fi + r] = accW[e];
        else if (r == Fi) row[o + H * Fi + c] = accW[e];
      }
    }
  }
  for (int blk = 0; blk < a.n_blocks; ++blk) {
    const int Fi = blk == 0 ? a.Fin : H, o = cl_block_offset(blk, a.Fin, H) + 2 * H * Fi + 2 * H;
    for (int which = 0; which < 2; ++which) {  // att, bias
      __syncthreads();
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        if (blk == 1) {
          const float v = lg_row_parity_sum(which == 0 ? gatt1[k] : gbias1[k]);
          if ((lane & 14) == 14) red[(tid >> 4) * 32 + c0 + k] = v;
        }
      }
      __syncthreads();
      if (tid < H) {
        float s = 0.f;
        if (blk == 1) {
#pragma unroll 8
          for (int w = 0; w < kLgRows; ++w) s += red[w * 32 + tid];
        } else {
          s = reinterpret_cast<const float*>(lds + m.acc0)[which * 32 + tid];
        }
        row[o + which * H + tid] = s;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static LgLayout lg_layout(const ClArgs& a, int HV, bool bwd) {
  LgLayout m{};
  m.P = a.P;
  m.P32 = (a.P + 31) & ~31;
  m.PK = (a.P + 15) & ~15;
  m.RS = HV + 4;   // 16 B x odd: the per-message row gathers spread over the bank quads
  m.TS = m.PK + 8;
  m.L = a.L;
  m.nslots = bwd ? (a.L >= 2 ? a.L - 1 : 1) : 1;
  m.xs = bwd ? (a.L >= 2 ? a.L - 2 : 0) : 0;
  int o = 0;
  auto take = [&](long bytes) {
    const int at = o;
    o += (int)((bytes + 15) & ~15L);
    return at;
  };
  const int M = a.M;
  m.frag = take((bwd ? 3 : 2) * 4 * 64 * 16);
  m.vec = take(2 * kMfVec * 4);
  m.ord = take(2 * m.P * 2);
  m.iptr = take((m.P + 1) * 4);
  m.deg = take(m.P * 4);
  m.isrc = take(M * 2);
  if (bwd) {
    m.optr = take((m.P + 1) * 4);
    m.oq = take(M * 2);
    m.odst = take(M * 2);
    m.sc = take(M * 4);
    m.ds = take(M * 4);
    m.zb = take(M * 4);
  }
  for (int s = 0; s < m.nslots; ++s) m.slot[s] = take(m.P32 * kMfRS * 2);
  const long fb = ((long)m.P * m.RS * 4 + 15) & ~15L;
  const long dt = 32L * m.TS * 2, dn = (long)m.P32 * kMfRS * 2;
  const long rsz = bwd ? (3 * fb > 2 * dt + 2 * dn ? 3 * fb : 2 * dt + 2 * dn) : 2 * fb;
  m.R = take(rsz);
  m.xl = m.R;
  m.xr = m.R + (int)fb;
  m.dy = m.R + 2 * (int)fb;
  m.dtl = m.R;
  m.dtr = m.R + (int)dt;
  m.dnl = m.R + 2 * (int)dt;
  m.dnr = m.R + 2 * (int)dt + (int)dn;
  if (bwd) m.ht = take(dt);
  m.red = take(kLgRows * 32 * 4);
  if (bwd) m.acc0 = take(64 * 4);
  m.total = o;
  return m;
}

// GSC_LG_PROF=1: the phase-clock kernel variants accumulate into a 32-word device buffer (gnn_lg_prof reads and
// clears it: [0..5] forward phases, [16..28] backward phases, workgroup-summed shader cycles)
static bool lg_prof_on() {
  const char* e = getenv("GSC_LG_PROF");
  if (!(e && e[0] == '1')) return false;
  if (!g_lg_prof) {
    GSC_HIP_CHECK(hipMalloc(&g_lg_prof, 32 * sizeof(unsigned long long)));
    GSC_HIP_CHECK(hipMemset(g_lg_prof, 0, 32 * sizeof(unsigned long long)));
  }
  return true;
}
std::vector<unsigned long long> gnn_lg_prof() {
  std::vector<unsigned long long> v(32, 0);
  if (g_lg_prof) {
    GSC_HIP_CHECK(hipMemcpy(v.data(), g_lg_prof, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    GSC_HIP_CHECK(hipMemset(g_lg_prof, 0, 32 * sizeof(unsigned long long)));
  }
  return v;
}

static int lg_hv(int H) { return H < 16 ? 16 : (H < 24 ? 24 : 32); }  // H < HV: channel HV - 1 free for u / v

bool gnn_lg_supported(int Fin, int H, int NM, int P, int M, int L, int n_blocks, const int* layer_of) {
  // encoder + one shared process block, >= 2 convs (no ReLU after the last), bias gradients from a ones row of
  // the augmented dW product (F_in, H < 32), node ids / message positions as u16
  if (!(Fin >= 1 && Fin <= 16 && H >= 1 && H <= 31 && NM > 64 && P >= NM && P <= kLgMaxNodes && M <= 8192 && L >= 2 &&
        L <= kClMaxLayers && n_blocks == 2))
    return false;
  for (int l = 0; l < L; ++l)
    if ((l == 0) != (layer_of[l] == 0)) return false;
  ClArgs a{};
  a.Fin = Fin; a.H = H; a.NM = NM; a.M = M; a.P = P; a.L = L; a.n_blocks = n_blocks;
  const int HV = lg_hv(H);
  return lg_layout(a, HV, false).total <= 160 * 1024 && lg_layout(a, HV, true).total <= 160 * 1024;
}

template <int HV>
static void lg_launch_fwd(const ClArgs& a, hipStream_t st, int cus) {
  const LgLayout m = lg_layout(a, HV, false);
  const size_t lds = m.total;
  GSC_CHECK(lds <= 160 * 1024, "GNN (large-graph fused) forward working set exceeds LDS");
  const bool prof = lg_prof_on();
  const void* fn = prof ? (const void*)gnn_lg_fwd_kernel<HV, true> : (const void*)gnn_lg_fwd_kernel<HV, false>;
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu > 2 ? 2 : (per_cu < 1 ? 1 : per_cu);
  long grid = (long)cus * per_cu;
  if (grid > a.B) grid = a.B;
  if (grid < 1) grid = 1;
  if (prof) hipLaunchKernelGGL((gnn_lg_fwd_kernel<HV, true>), dim3((unsigned)grid), dim3(kLgThreads), lds, st, a, m, g_lg_prof);
  else hipLaunchKernelGGL((gnn_lg_fwd_kernel<HV, false>), dim3((unsigned)grid), dim3(kLgThreads), lds, st, a, m, nullptr);
  check_launch();
}

template <int HV>
static int lg_launch_bwd(const ClArgs& a, hipStream_t st, int cus, int max_rows) {
  const LgLayout m = lg_layout(a, HV, true);
  const size_t lds = m.total;
  GSC_CHECK(lds <= 160 * 1024, "GNN (large-graph fused) backward working set exceeds LDS");
  const bool prof = lg_prof_on();
  const void* fn = prof ? (const void*)gnn_lg_bwd_kernel<HV, true> : (const void*)gnn_lg_bwd_kernel<HV, false>;
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long grid = cus;
  if (grid > a.B) grid = a.B;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  if (prof) hipLaunchKernelGGL((gnn_lg_bwd_kernel<HV, true>), dim3((unsigned)grid), dim3(kLgThreads), lds, st, a, m, g_lg_prof);
  else hipLaunchKernelGGL((gnn_lg_bwd_kernel<HV, false>), dim3((unsigned)grid), dim3(kLgThreads), lds, st, a, m, nullptr);
  check_launch();
  return (int)grid;
}

static void lg_check(const ClArgs& a) {
  GSC_CHECK(a.P <= kLgMaxNodes && a.P >= a.NM && a.M <= 8192 && a.H <= 31 && a.Fin <= 16 && a.L >= 2 && a.n_blocks == 2,
            "large-graph fused GNN: shape outside the kernel's assumptions (gnn_lg_supported)");
}

void gnn_lg_forward(const void* args_generic, uintptr_t stream, int cus) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  lg_check(a);
  switch (lg_hv(a.H)) {
    case 16: lg_launch_fwd<16>(a, stream_of(stream), cus); break;
    case 24: lg_launch_fwd<24>(a, stream_of(stream), cus); break;
    default: lg_launch_fwd<32>(a, stream_of(stream), cus); break;
  }
}

int gnn_lg_backward(const void* args_generic, uintptr_t stream, int cus, int max_rows) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  lg_check(a);
  switch (lg_hv(a.H)) {
    case 16: return lg_launch_bwd<16>(a, stream_of(stream), cus, max_rows);
    case 24: return lg_launch_bwd<24>(a, stream_of(stream), cus, max_rows);
    default: return lg_launch_bwd<32>(a, stream_of(stream), cus, max_rows);
  }
}

}  // namespace gsc
