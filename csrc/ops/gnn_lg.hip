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
constexpr int kLgBwdThreads = 1024;  // backward: 16 waves, 4 lanes per node
constexpr float kLgSlope = 0.2f;
constexpr int kLgUf = 2;  // messages per chunk in the forward attention loop (registers: 4 waves / SIMD)
constexpr int kLgUb = 2;  // ... in the backward's row-reading loops

struct LgLayout {
  int P, P32, PK, RS, TS, L, nslots, xs;
  int G, NP, gm, nv;  // graphs per pack (one workgroup's unit of work), nodes per graph (n_pad), pack meta, node valid
  int frag, vec, ord, iptr, deg, isrc, optr, oq, odst, sc, ds, zb, slot[kClMaxLayers], R, xl, xr, dy, dtl, dtr, dnl, dnr, ht,
      red, acc0, wacc, wq, total;
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


// Lane groups: NL consecutive lanes (2 or 4) hold one node, HV / NL channels each.
// Sum over the node's NL lanes (the score's / dalpha's channel sum): DPP quad permutations, no LDS
template <int NL>
__device__ __forceinline__ float lg_node_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  if (NL == 4) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  return v;
}
// Sum over the wave's nodes of one channel slot (lanes of the same position within their group): DPP row
// shifts within each 16-lane row, then the four rows; complete in the wave's last NL lanes (lanes 64-NL .. 63)
template <int NL>
__device__ __forceinline__ float lg_wave_sum(float v) {
  if (NL <= 2) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));  // row_shr:2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false));  // row_shr:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false));  // row_shr:8
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int HC>
__device__ __forceinline__ void lg_load_f(float (&v)[HC], const float* src) {  // 16-B (HC % 4 == 0) or 8-B runs
  if constexpr (HC % 4 == 0) {
#pragma unroll
    for (int u = 0; u < HC / 4; ++u) {
      const float4 f = reinterpret_cast<const float4*>(src)[u];
      v[4 * u] = f.x;
      v[4 * u + 1] = f.y;
      v[4 * u + 2] = f.z;
      v[4 * u + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < HC / 2; ++u) {
      const float2 f = reinterpret_cast<const float2*>(src)[u];
      v[2 * u] = f.x;
      v[2 * u + 1] = f.y;
    }
  }
}
template <int HC>
__device__ __forceinline__ void lg_store_f(float* dst, const float (&v)[HC]) {
  if constexpr (HC % 4 == 0) {
#pragma unroll
    for (int u = 0; u < HC / 4; ++u)
      reinterpret_cast<float4*>(dst)[u] = float4{v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]};
  } else {
#pragma unroll
    for (int u = 0; u < HC / 2; ++u) reinterpret_cast<float2*>(dst)[u] = float2{v[2 * u], v[2 * u + 1]};
  }
}
template <int HC>
__device__ __forceinline__ void lg_store_bf16(__bf16* dst, const float (&v)[HC]) {  // 8-B or 4-B stores
  if constexpr (HC % 4 == 0) {
#pragma unroll
    for (int u = 0; u < HC / 4; ++u) {
      bf16x4 b;
#pragma unroll
      for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[4 * u + e];
      reinterpret_cast<bf16x4*>(dst)[u] = b;
    }
  } else {
#pragma unroll
    for (int u = 0; u < HC / 2; ++u) {
      __attribute__((ext_vector_type(2))) __bf16 b;
      b[0] = (__bf16)v[2 * u];
      b[1] = (__bf16)v[2 * u + 1];
      reinterpret_cast<decltype(b)*>(dst)[u] = b;
    }
  }
}
template <int HC>
__device__ __forceinline__ void lg_load_bf16(float (&v)[HC], const __bf16* src) {
  if constexpr (HC % 4 == 0) {
#pragma unroll
    for (int u = 0; u < HC / 4; ++u) {
      const bf16x4 b = reinterpret_cast<const bf16x4*>(src)[u];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * u + e] = (float)b[e];
    }
  } else {
#pragma unroll
    for (int u = 0; u < HC / 2; ++u) {
      const __attribute__((ext_vector_type(2))) __bf16 b = reinterpret_cast<const __attribute__((ext_vector_type(2))) __bf16*>(src)[u];
      v[2 * u] = (float)b[0];
      v[2 * u + 1] = (float)b[1];
    }
  }
}

// Weight fragments of the node linears (set 2b: block b, B operand of h W^T) and of the input gradient (set
// 2: block 1 transposed, B operand of dX W), lane-linear in LDS: [set][Wl k-step 0, 1, Wr k-step 0, 1][lane]
__device__ __forceinline__ void lg_stage_frags(const ClArgs& a, bf16x8* img, int nsets) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int f = wave; f < nsets; f += blockDim.x / 64) {
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
// rescale per chunk) and mean aggregation; returns the conv output half-row (bias, optional ReLU; zero unless real).
// Messages go U at a time: the U source ids, then the U rows are loaded before any of them is used (clamped to
// the segment's last message), so one LDS round trip serves U messages.
template <int HC, int U, int NL>
__device__ __forceinline__ void lg_attend(float (&y)[HC], int i, bool real, int c0, bool hi, const float* vec, bool relu,
                                          const float* XL, const float* XR, const int32_t* iptr,
                                          const uint16_t* isrc, const float* deg, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) y[k] = 0.f;
  if (!real) return;
  // score = att . LeakyReLU(z) = 0.6 (u_j + v_i) + 0.4 att . |z|: one FMA per channel with the |z| source
  // modifier; the lane holding channel HV - 1 (u + v; hi) adds the linear part
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
      v = lg_node_sum<NL>(v);
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

// Topology rows of pack pk's graphs into LDS (u16 message arrays; the backward also the source-sorted CSR).  A pack
// is G consecutive batch entries b0 .. b0 + G - 1 laid out as one disjoint graph of G x NP nodes: graph g's node v
// is node g NP + v and its messages follow graph g - 1's (offsets in the pack meta).  Graphs past the batch are
// empty (no real nodes, no messages).  G = 1 (200 nodes): the topology of b0 as is.  Lane-pair order interleaves
// the graphs (rank p -> graph p mod G, that graph's node of degree rank p / G): every wave gets a similar mix.
// Pack meta (LDS ints): [0, 8) topology (-1: empty), [8, 16) real nodes, [16, 25) message offsets.
template <bool BWD, int NT, bool PK>
__device__ __forceinline__ void lg_stage_topo(const ClArgs& a, long b0, int t1, int n1, char* lds, const LgLayout& m) {
  int32_t* iptr = reinterpret_cast<int32_t*>(lds + m.iptr);
  float* deg = reinterpret_cast<float*>(lds + m.deg);
  uint16_t* isrc = reinterpret_cast<uint16_t*>(lds + m.isrc);
  uint16_t* ord = reinterpret_cast<uint16_t*>(lds + m.ord);
  uint8_t* nv = reinterpret_cast<uint8_t*>(lds + m.nv);
  int* gm = reinterpret_cast<int*>(lds + m.gm);
  const int P = m.P, NP = m.NP, G = PK ? m.G : 1, M = a.M;
  if constexpr (!PK) {  // one graph (topology t1, n1 nodes: loaded by the caller before its barrier): its tables as they are
    const int t = t1;
    if (threadIdx.x == 0) gm[8] = n1;  // (the pooling's node count; validity is u < n1 in registers)
    for (int k = threadIdx.x; k < 2 * P; k += NT) ord[k] = (uint16_t)a.deg_order[(long)t * 2 * P + k];
    for (int k = threadIdx.x; k <= P; k += NT) {
      iptr[k] = a.in_ptr[(long)t * (P + 1) + k];
      if (k < P) deg[k] = a.deg[(long)t * P + k];
      if (BWD) reinterpret_cast<int32_t*>(lds + m.optr)[k] = a.out_ptr[(long)t * (P + 1) + k];
    }
    for (int k = threadIdx.x; k < M; k += NT) {
      isrc[k] = (uint16_t)a.in_src[(long)t * M + k];
      if (BWD) {
        reinterpret_cast<uint16_t*>(lds + m.oq)[k] = (uint16_t)a.out_q[(long)t * M + k];
        reinterpret_cast<uint16_t*>(lds + m.odst)[k] = (uint16_t)a.out_dst[(long)t * M + k];
      }
    }
    return;
  }
  if (threadIdx.x == 0) {
    int off = 0;
    for (int g = 0; g < G; ++g) {
      const long b = b0 + g;
      const int t = b < a.B ? a.topo[b] : -1;
      gm[g] = t;
      gm[8 + g] = t >= 0 ? a.nnodes[t] : 0;
      gm[16 + g] = off;
      off += t >= 0 ? a.in_ptr[(long)t * (NP + 1) + NP] : 0;
    }
    gm[16 + G] = off;
  }
  __syncthreads();
  const int total = gm[16 + G];
  for (int k = threadIdx.x; k < 2 * P; k += NT) {
    const int half = k >= P, p = k - half * P, g = p % G, r = p / G, t = gm[g];
    ord[k] = (uint16_t)(g * NP + (t >= 0 ? a.deg_order[(long)t * 2 * NP + half * NP + r] : r));
  }
  for (int u = threadIdx.x; u <= P; u += NT) {
    if (u == P) {
      iptr[P] = total;
      if (BWD) reinterpret_cast<int32_t*>(lds + m.optr)[P] = total;
      continue;
    }
    const int g = u / NP, v = u - g * NP, t = gm[g], o = gm[16 + g];
    iptr[u] = o + (t >= 0 ? a.in_ptr[(long)t * (NP + 1) + v] : 0);
    deg[u] = t >= 0 ? a.deg[(long)t * NP + v] : 1.f;
    nv[u] = (uint8_t)(v < gm[8 + g]);
    if (BWD) reinterpret_cast<int32_t*>(lds + m.optr)[u] = o + (t >= 0 ? a.out_ptr[(long)t * (NP + 1) + v] : 0);
  }
  for (int k = threadIdx.x; k < total; k += NT) {
    int g = 0;
    while (g + 1 < G && k >= gm[16 + g + 1]) ++g;
    const int t = gm[g], o = gm[16 + g], q = k - o;
    isrc[k] = (uint16_t)(g * NP + a.in_src[(long)t * M + q]);
    if (BWD) {
      reinterpret_cast<uint16_t*>(lds + m.oq)[k] = (uint16_t)(o + a.out_q[(long)t * M + q]);
      reinterpret_cast<uint16_t*>(lds + m.odst)[k] = (uint16_t)(g * NP + a.out_dst[(long)t * M + q]);
    }
  }
}

// node u of the pack is a real node (not padding, not an empty graph's); G = 1: u < n1, the graph's node count
template <bool PK>
__device__ __forceinline__ bool lg_real(const char* lds, const LgLayout& m, int u, int n1) {
  if constexpr (!PK) return u < n1;
  return u < m.P && reinterpret_cast<const uint8_t*>(lds + m.nv)[u] != 0;
}

// input rows of pack node i (graph b0 + i / NP, node i mod NP) as the bf16 image (channels 0..15: F_in <= 16, zero
// past F_in, for rows >= P and for graphs past the batch)
// (g = the lane's position in its node group: lanes 0 / 1 of the group take channels 0..7 / 8..15)
template <bool PK>
__device__ __forceinline__ void lg_load_x(float (&xv)[8], const ClArgs& a, const LgLayout& m, long b0, int i, int g) {
  const int gi = PK ? i / m.NP : 0, v = i - gi * m.NP;
  const long b = b0 + gi;
  const bool ok = i < m.P && g < 2 && b < a.B;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = 8 * g + k;
    xv[k] = (ok && c < a.Fin) ? a.x[(b * m.NP + v) * a.Fin + c] : 0.f;
  }
}
__device__ __forceinline__ void lg_put_x(__bf16* S, const float (&xv)[8], int i, int hf, const LgLayout& m) {
  if (i < m.P32 && hf < 2) {
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (__bf16)xv[k];
    *reinterpret_cast<bf16x8*>(S + i * kMfRS + 8 * hf) = v;
  }
}

// Next graph of this workgroup (every thread calls; one barrier): fixed stride, or -- a.work set (overlap mode: a
// zeroed counter, full-device grid) -- claimed from the counter, so CUs the simulator frees mid-kernel join in
// (per-workgroup gradient rows then depend on the claim order: summation order, not values, varies)
__device__ __forceinline__ long lg_next_graph(const ClArgs& a, int* slot, long cur) {
  if (threadIdx.x == 0) *slot = a.work ? atomicAdd(a.work, 1) : (int)(cur < 0 ? (long)blockIdx.x : cur + gridDim.x);
  __syncthreads();
  return *slot;
}

__device__ __forceinline__ void lg_zero(char* p, int bytes) {
  for (int k = 16 * threadIdx.x; k < bytes; k += 16 * blockDim.x) *reinterpret_cast<float4*>(p + k) = float4{0, 0, 0, 0};
}

// ---------------------------------------------------------------------------------------------
// forward: emb[b] = mean over real nodes of the last conv's rows (a.params2 / a.emb2: unused here; two launches)
// ---------------------------------------------------------------------------------------------
template <int HV, bool PROF, bool PK>
__global__ __launch_bounds__(kLgThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void gnn_lg_fwd_kernel(ClArgs a, LgLayout m, unsigned long long* prof) {
  constexpr int NL = 2, HC = HV / NL;  // lane pairs: 2 workgroups of 8 waves per CU
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
  int* wq = reinterpret_cast<int*>(lds + m.wq);
  const int G = PK ? m.G : 1;  // graphs per pack (PK: packs of small graphs; else one graph per workgroup)
  const long npk = (a.B + G - 1) / G;
  for (long pk = lg_next_graph(a, wq, -1); pk < npk; pk = lg_next_graph(a, wq, pk)) {
    const long b0 = pk * G;
    const int t1 = a.topo[b0], n1 = a.nnodes[t1];  // (G = 1: the staging's topology, loaded before the barrier)
    {
      const int tq = lg_tid();
      float xv[8];
      lg_load_x<PK>(xv, a, m, b0, tq / NL, tq % NL);
      __syncthreads();  // the previous pack is done with every LDS image
      LG_MARK(PROF, clk, 0);
      lg_stage_topo<false, kLgThreads, PK>(a, b0, t1, n1, lds, m);
      lg_put_x(S, xv, tq / NL, tq % NL, m);
      __syncthreads();
      LG_MARK(PROF, clk, 1);
    }
    const int32_t* iptr = reinterpret_cast<const int32_t*>(lds + m.iptr);
    const uint16_t* isrc = reinterpret_cast<const uint16_t*>(lds + m.isrc);
    const float* deg = reinterpret_cast<const float*>(lds + m.deg);
    const int* gm = reinterpret_cast<const int*>(lds + m.gm);
    for (int l = 0; l < a.L; ++l) {
      const int blk = a.layer_of[l];
      const float* vb = vec + blk * kMfVec;
      lg_linear<HV>(frag, blk, blk ? k2b : false, vb, S, XL, XR, m);
      __syncthreads();
      LG_MARK(PROF, clk, 2);
      // lane pair p = the node of in-degree rank p (similar segment lengths per wave); p >= P: idle (zero rows)
      const int tq = lg_tid(), pq = tq / NL, cq = (tq % NL) * HC, lane = tq & 63;
      const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
      float y[HC];
      const bool last = l + 1 == a.L;
      lg_attend<HC, kLgUf, NL>(y, iq, lg_real<PK>(lds, m, iq, n1), cq, cq + HC == HV, vb, !last, XL, XR, iptr, isrc, deg, m);
      if (!last) {
        __syncthreads();  // S (this conv's input) was read by the node linears before the previous barrier;
                          // the barrier orders this conv's XL reads before the next node linears' XL writes
        LG_MARK(PROF, clk, 3);
        if (iq < m.P32) lg_store_bf16<HC>(S + iq * kMfRS + cq, y);
        __syncthreads();
        LG_MARK(PROF, clk, 4);
      } else if (!PK) {  // mean pool over the real nodes: wave sums (DPP + two swaps), then the waves in a fixed order
#pragma unroll
        for (int k = 0; k < HC; ++k) {
          const float v = lg_wave_sum<NL>(y[k]);  // y is zero for nodes that are not real
          if (lane >= 64 - NL) red[wave * 32 + cq + k] = v;
        }
        __syncthreads();
        if (tq < a.H && b0 < a.B) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < kLgThreads / 64; ++w) s += red[w * 32 + tq];
          a.emb[b0 * a.H + tq] = s / (float)gm[8];
        }
        LG_MARK(PROF, clk, 5);
      } else {  // packs: the rows into LDS (XR is dead), then one thread per (graph, channel) sums its graph's rows
        __syncthreads();  // every lane's XR reads are done
        if (iq < m.P) lg_store_f<HC>(XR + iq * m.RS + cq, y);
        __syncthreads();
        if (tq < G * a.H) {
          const int g = tq / a.H, c = tq - g * a.H, n = gm[8 + g];
          float s = 0.f;
          for (int v = 0; v < n; ++v) s += XR[(g * m.NP + v) * m.RS + c];
          if (n > 0) a.emb[(b0 + g) * a.H + c] = s / (float)n;
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
// step 2: per target node i -- softmax backward and d x_r[i]; alpha / d score per message into SC / DS.
//   d x_r[i] = att * sum_q ds_q LeakyReLU'(z_q),  ds_q = alpha_q (dalpha_q - c),  c = sum_q alpha_q dalpha_q
// With LeakyReLU'(z) = 0.2 + 0.8 [z > 0] and sum_q ds_q = 0 this is 0.8 att * (T1 - c T2) / den, where
// T1 = sum_q e_q dalpha_q [z_q > 0] and T2 = sum_q e_q [z_q > 0] accumulate (online-rescaled, like the forward's
// aggregation) in the same pass over the source rows that forms the scores and dalpha = dY_i . x_l[j] / deg_i --
// no per-message sign bits, no second row pass.  A row-free pass then writes alpha and ds for step 3.
// [z > 0] is saturate(z * 2^126): exact except for denormal z.
template <int HC, int U, int NL>
__device__ __forceinline__ void lg_bwd_targets(float (&dxr)[HC], float (&gbias)[HC], int i, bool real, int c0, bool hi,
                                               const float* vec, char* lds, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) dxr[k] = 0.f;
  if (!real) return;
  const float* XL = reinterpret_cast<const float*>(lds + m.xl);
  const float* XR = reinterpret_cast<const float*>(lds + m.xr);
  const float* DY = reinterpret_cast<const float*>(lds + m.dy);
  const int32_t* iptr = reinterpret_cast<const int32_t*>(lds + m.iptr);
  const uint16_t* isrc = reinterpret_cast<const uint16_t*>(lds + m.isrc);
  const float* deg = reinterpret_cast<const float*>(lds + m.deg);
  float* SC = reinterpret_cast<float*>(lds + m.sc);
  float* DS = reinterpret_cast<float*>(lds + m.ds);
  float xr[HC], a4[HC], dy[HC], t1[HC], t2[HC];
  lg_load_f<HC>(xr, XR + i * m.RS + c0);
  lg_load_f<HC>(a4, vec + 64 + c0);
  lg_load_f<HC>(dy, DY + i * m.RS + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    gbias[k] += dy[k];
    a4[k] *= 0.5f * (1.f - kLgSlope);
    t1[k] = t2[k] = 0.f;
  }
  const int q0 = iptr[i], q1 = iptr[i + 1];
  const float rdeg = 1.f / deg[i];
  const float lin = hi ? 0.5f * (1.f + kLgSlope) : 0.f;  // the lane holding channel HV - 1 (u + v): linear part
  const bool lead = c0 == 0;  // the group's first lane writes the per-message scalars
  float mx = -__builtin_inff(), den = 0.f, ced = 0.f;  // ced = sum e dalpha
  for (int q = q0; q < q1; q += U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = isrc[min(q + u, q1 - 1)];
    float xj[U][HC];
#pragma unroll
    for (int u = 0; u < U; ++u) lg_load_f<HC>(xj[u], XL + j[u] * m.RS + c0);
    float sc[U], da[U];
    float cm = -__builtin_inff();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v = lin * (xj[u][HC - 1] + xr[HC - 1]), d = 0.f;
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        v = fmaf(a4[k], fabsf(xj[u][k] + xr[k]), v);
        d = fmaf(dy[k], xj[u][k], d);
      }
      v = lg_node_sum<NL>(v);
      d = lg_node_sum<NL>(d);
      sc[u] = q + u < q1 ? v : -__builtin_inff();
      da[u] = d * rdeg;
      cm = fmaxf(cm, sc[u]);
    }
    if (cm > mx) {
      const float rs = __expf(mx - cm);  // 0 for the first chunk
      den *= rs;
      ced *= rs;
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        t1[k] *= rs;
        t2[k] *= rs;
      }
      mx = cm;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float e = __expf(sc[u] - mx), ed = e * da[u];  // 0 past the segment
      den += e;
      ced += ed;
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        const float st = __saturatef((xj[u][k] + xr[k]) * 0x1p126f);
        t1[k] = fmaf(ed, st, t1[k]);
        t2[k] = fmaf(e, st, t2[k]);
      }
      if (q + u < q1 && lead) {
        SC[q + u] = sc[u];
        DS[q + u] = da[u];
      }
    }
  }
  const float inv = 1.f / (den + 1e-16f), cs = ced * inv;
#pragma unroll
  for (int k = 0; k < HC; ++k)  // 0.8 att = 2 a4 (a4 = 0.4 att)
    dxr[k] = 2.f * a4[k] * (t1[k] - cs * t2[k]) * inv;
  // alpha and ds per message (the group's lead lane wrote this wave's SC / DS entries: program order)
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
      if (q + u < q1 && lead) {
        SC[q + u] = al;
        DS[q + u] = al * (dv[u] - cs);
      }
    }
  }
}

// step 3: per source node j through the source-sorted CSR -- d x_l[j] and the attention-vector gradient (U
// out-messages at a time: ids, then the target rows of x_r and dY, all loaded before use)
template <int HC, int U>
__device__ __forceinline__ void lg_bwd_sources(float (&dxl)[HC], float (&gatt)[HC], int j, bool real, int c0,
                                               const float* vec, char* lds, const LgLayout& m) {
#pragma unroll
  for (int k = 0; k < HC; ++k) dxl[k] = 0.f;
  if (!real) return;
  const float* XL = reinterpret_cast<const float*>(lds + m.xl);
  const float* XR = reinterpret_cast<const float*>(lds + m.xr);
  const float* DY = reinterpret_cast<const float*>(lds + m.dy);
  const int32_t* optr = reinterpret_cast<const int32_t*>(lds + m.optr);
  const uint16_t* oq = reinterpret_cast<const uint16_t*>(lds + m.oq);
  const uint16_t* odst = reinterpret_cast<const uint16_t*>(lds + m.odst);
  const float* deg = reinterpret_cast<const float*>(lds + m.deg);
  const float* SC = reinterpret_cast<const float*>(lds + m.sc);
  const float* DS = reinterpret_cast<const float*>(lds + m.ds);
  // d x_l[j] = sum_p w_p dY_i + att * sum_p ds_p LeakyReLU'(z_p) = sum_p w_p dY_i + att * (0.2 S + 0.8 T),
  // S = sum_p ds_p, T = sum_p ds_p [z_p > 0];  d att += sum_p ds_p LeakyReLU(z_p) = 0.6 ds z + 0.4 ds |z|
  float xl[HC], tt[HC], sds = 0.f;
  lg_load_f<HC>(xl, XL + j * m.RS + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) tt[k] = 0.f;
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
      const bool ok = p + u < p1;
      w[u] = ok ? SC[q[u]] / deg[ti[u]] : 0.f;
      ds[u] = ok ? DS[q[u]] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float d6 = 0.5f * (1.f + kLgSlope) * ds[u], d4 = 0.5f * (1.f - kLgSlope) * ds[u];
      sds += ds[u];
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        const float z = xl[k] + xr[u][k];
        gatt[k] = fmaf(d6, z, fmaf(d4, fabsf(z), gatt[k]));
        tt[k] = fmaf(ds[u], __saturatef(z * 0x1p126f), tt[k]);
        dxl[k] = fmaf(w[u], dy[u][k], dxl[k]);
      }
    }
  }
  float at[HC];
  lg_load_f<HC>(at, vec + 64 + c0);
#pragma unroll
  for (int k = 0; k < HC; ++k) dxl[k] = fmaf(at[k], fmaf(1.f - kLgSlope, tt[k], kLgSlope * sds), dxl[k]);
}

// dst[k] += sum over the wave's nodes of v[k] (this lane's HC channels; dst points at the lane's first channel in
// the wave's own slot): wave sums, then the wave's last node group adds -- one writer per slot, fixed order
template <int HC, int NL>
__device__ __forceinline__ void lg_wave_accum(float* dst, const float (&v)[HC], int lane) {
  float s[HC];
#pragma unroll
  for (int k = 0; k < HC; ++k) s[k] = lg_wave_sum<NL>(v[k]);
  if (lane >= 64 - NL) {
#pragma unroll
    for (int k = 0; k < HC; ++k) dst[k] += s[k];
  }
}

// HT [k][node] (bf16, row stride TS) of the conv input image S: channels < Fi, a ones row at k = Fi (bias
// gradients from the same product), zero rows in between up to HV; zero columns for nodes >= P
template <int HC, int HV>
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
  if (Fi >= HV && c0 + HC == HV) HT[Fi * m.TS + i] = (__bf16)(i < m.P ? 1.f : 0.f);  // ones row past the channels
}

template <int HV, int NL, bool PROF, bool PK>
__global__ __launch_bounds__(256 * NL) void gnn_lg_bwd_kernel(ClArgs a, LgLayout m, unsigned long long* prof) {
  // node groups of NL lanes (HV / NL channels each).  NL = 4: 16 waves, so the one workgroup an LDS-full CU holds
  // still has 4 waves per SIMD to hide the message loops' LDS latency
  constexpr int HC = HV / NL, NT = 256 * NL;
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
  // gradient accumulators over all the graphs of this workgroup: per lane (attention vector, output bias; HC
  // channels of a node) and, in waves 0..3, the augmented weight gradients [dW | db] of (block, side)
  // (block 1, convs 1 .. L-1: registers for the workgroup's whole run; block 0, conv 0 only: per graph, then
  // summed over the wave's nodes into the wave's own LDS slot -- 24 fewer live registers)
  // per-wave [block][att | bias][32] sums over the workgroup's graphs (each wave owns its slots: no barrier)
  for (int k = threadIdx.x; k < NT / 64 * 128; k += NT) reinterpret_cast<float*>(lds + m.wacc)[k] = 0.f;
  f32x16 accW;
  mf_zero(accW);
  const int wblk = wave >> 1, wside = wave & 1;  // waves 0..3: (block, l | r) of accW
  LgClock clk{};
  if (PROF) clk.last = __builtin_amdgcn_s_memtime();
  int* wq = reinterpret_cast<int*>(lds + m.wq);
  const int G = PK ? m.G : 1;  // graphs per pack (PK: packs of small graphs; else one graph per workgroup)
  const long npk = (a.B + G - 1) / G;
  for (long pk = lg_next_graph(a, wq, -1); pk < npk; pk = lg_next_graph(a, wq, pk)) {
    const long b0 = pk * G;
    const int t1 = a.topo[b0], n1 = a.nnodes[t1];  // (G = 1: the staging's topology, loaded before the barrier)
    {
      const int tq = lg_tid(), iq = tq / NL, hq = tq % NL, cq = hq * HC;
      float xv[8], dy0[HC];
      lg_load_x<PK>(xv, a, m, b0, iq, hq);
      // d emb / n on every real node of the node's graph (L >= 2: no ReLU after the last conv); G = 1: loaded
      // before the barrier
      if (!PK) {  // raw loads (no dependence on n1: they overlap the barrier), masked after it
#pragma unroll
        for (int k = 0; k < HC; ++k) dy0[k] = a.demb[b0 * a.H + min(cq + k, a.H - 1)];
      }
      __syncthreads();  // the previous pack is done with every LDS image
      LG_MARK(PROF, clk, 0);
      lg_stage_topo<true, NT, PK>(a, b0, t1, n1, lds, m);
      lg_put_x(reinterpret_cast<__bf16*>(lds + m.slot[m.xs]), xv, iq, hq, m);
      if (!PK) {
        const float rn = 1.f / (float)n1;
#pragma unroll
        for (int k = 0; k < HC; ++k) dy0[k] = (iq < n1 && cq + k < a.H) ? dy0[k] * rn : 0.f;
      }
      if (PK) {  // the node's graph from the pack meta (visible since lg_stage_topo's barrier)
        const int* gm = reinterpret_cast<const int*>(lds + m.gm);
        const int g = iq / m.NP, ng = gm[8 + g];
        const bool real = iq < m.P && iq - g * m.NP < ng;
        const float rn = real ? 1.f / (float)ng : 0.f;
#pragma unroll
        for (int k = 0; k < HC; ++k) dy0[k] = (real && cq + k < a.H) ? a.demb[(b0 + g) * a.H + cq + k] * rn : 0.f;
      }
      if (iq < m.P) lg_store_f<HC>(DY + iq * m.RS + cq, dy0);
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
      const int tq = lg_tid(), pq = tq / NL, cq = (tq % NL) * HC;
      const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
      float y[HC];
      lg_attend<HC, kLgUb, NL>(y, iq, lg_real<PK>(lds, m, iq, n1), cq, cq + HC == HV, vb, true, XL, XR, iptr, isrc, deg, m);
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
        lg_load_x<PK>(xv, a, m, b0, tq / NL, tq % NL);
        lg_put_x(Sin, xv, tq / NL, tq % NL, m);
        __syncthreads();
        LG_MARK(PROF, clk, 5);
      }
      // 1: x_l, x_r and HT
      lg_linear<HV>(frag, blk, blk ? k2b : false, vb, Sin, XL, XR, m);
      {
        const int tq = lg_tid();
        lg_put_ht<HC, HV>(HT, Sin, tq / NL, (tq % NL) * HC, Fi, m);
      }
      __syncthreads();
      LG_MARK(PROF, clk, 6);
      // 2 + 3
      // node group p: step 2's target = the node of in-degree rank p, step 3's source = the node of out-degree rank p
      float dxr[HC], dxl[HC], gv[HC];  // gv: this conv's bias, then attention-vector gradient (this lane's share)
      {
        const int tq = lg_tid(), pq = tq / NL, cq = (tq % NL) * HC;
        const int iq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[pq] : pq;
#pragma unroll
        for (int k = 0; k < HC; ++k) gv[k] = 0.f;
        lg_bwd_targets<HC, kLgUb, NL>(dxr, gv, iq, lg_real<PK>(lds, m, iq, n1), cq, cq + HC == HV, vb, lds, m);
        lg_wave_accum<HC, NL>(reinterpret_cast<float*>(lds + m.wacc) + (wave * 4 + 2 * blk + 1) * 32 + cq, gv, tq & 63);
      }
      __syncthreads();
      LG_MARK(PROF, clk, 7);
      {
        const int tq = lg_tid(), pq = tq / NL, cq = (tq % NL) * HC;
        const int jq = pq < m.P ? (int)reinterpret_cast<const uint16_t*>(lds + m.ord)[m.P + pq] : pq;
#pragma unroll
        for (int k = 0; k < HC; ++k) gv[k] = 0.f;
        lg_bwd_sources<HC, kLgUb>(dxl, gv, jq, lg_real<PK>(lds, m, jq, n1), cq, vb, lds, m);
        lg_wave_accum<HC, NL>(reinterpret_cast<float*>(lds + m.wacc) + (wave * 4 + 2 * blk) * 32 + cq, gv, tq & 63);
      }
      __syncthreads();  // XL / XR / DY are dead: their region takes DT / DN
      LG_MARK(PROF, clk, 8);
      // 4: d x_l, d x_r images
      __bf16* DTl = reinterpret_cast<__bf16*>(lds + m.dtl);
      __bf16* DTr = reinterpret_cast<__bf16*>(lds + m.dtr);
      __bf16* DNl = reinterpret_cast<__bf16*>(lds + m.dnl);
      __bf16* DNr = reinterpret_cast<__bf16*>(lds + m.dnr);
      {
        const int tq = lg_tid(), pq = tq / NL, cq = (tq % NL) * HC;
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
          if (cq + HC == HV) {  // K columns HV..31 of the dX product: zero (the region held fp32 rows)
#pragma unroll
            for (int c = HV; c < 32; c += 8) {
              *reinterpret_cast<bf16x8*>(DNl + jq * kMfRS + c) = bf16x8{};
              *reinterpret_cast<bf16x8*>(DNr + iq * kMfRS + c) = bf16x8{};
            }
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
    LG_MARK(PROF, clk, 12);
  }
  if (PROF && threadIdx.x == 0)
    for (int k = 0; k < 13; ++k) atomicAdd(prof + 16 + k, clk.ph[k]);
  // ---- this workgroup's gradient row (module layout per block: Wl, bl, Wr, br, att, bias)
  float* row = a.partials + (long)blockIdx.x * a.n_params;
  const int H = a.H;
  const int tid = threadIdx.x, c0 = (tid % NL) * HC, lane = tid & 63, r = lane & 31, hh = lane >> 5;
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
  __syncthreads();
  if (tid < H) {
    const float* wacc = reinterpret_cast<const float*>(lds + m.wacc);
    for (int blk = 0; blk < a.n_blocks; ++blk) {
      const int Fi = blk == 0 ? a.Fin : H, o = cl_block_offset(blk, a.Fin, H) + 2 * H * Fi + 2 * H;
      for (int which = 0; which < 2; ++which) {  // att, bias: the waves' slots in a fixed order
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += wacc[(w * 4 + 2 * blk + which) * 32 + tid];
        row[o + which * H + tid] = s;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static LgLayout lg_layout_g(const ClArgs& a, int HV, bool bwd, int G);
static int lg_hv(int H);

// graphs per pack: one graph of 65 .. 256 nodes, else the most n_pad-node graphs (<= 8, <= 256 lane groups) whose
// forward and backward working sets fit the CU's LDS (n_pad 50: 4 graphs = 200 nodes, as config 5's one graph)
static int lg_pack(const ClArgs& a) {
  if (a.P > 128) return 1;
  for (int G = (256 / a.P > 8 ? 8 : 256 / a.P); G > 1; --G) {
    if ((long)G * a.M > 8192) continue;
    const int HV = lg_hv(a.H);
    if (lg_layout_g(a, HV, false, G).total <= 160 * 1024 && lg_layout_g(a, HV, true, G).total <= 160 * 1024) return G;
  }
  return 1;
}

static LgLayout lg_layout(const ClArgs& a, int HV, bool bwd) { return lg_layout_g(a, HV, bwd, lg_pack(a)); }

static LgLayout lg_layout_g(const ClArgs& a, int HV, bool bwd, int G) {
  LgLayout m{};
  m.G = G;
  m.NP = a.P;
  m.P = m.G * a.P;
  m.P32 = (m.P + 31) & ~31;
  m.PK = (m.P + 15) & ~15;
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
  const int M = m.G * a.M;  // the pack's messages
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
  m.red = take((bwd ? kLgBwdThreads : kLgThreads) / 64 * 32 * 4);  // one 32-channel partial per wave
  m.wq = take(16);
  m.gm = take(25 * 4);
  m.nv = take(m.P);
  if (bwd) m.wacc = take(kLgBwdThreads / 64 * 128 * 4);
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

// GSC_GNN_LG_PACK=0: 33 .. 64-node graphs stay on the multi-tile kernels (gnn_mt.hip) instead of packs here
bool gnn_lg_pack_enabled() {
  const char* e = getenv("GSC_GNN_LG_PACK");
  return !(e && e[0] == '0');
}

bool gnn_lg_supported(int Fin, int H, int NM, int P, int M, int L, int n_blocks, const int* layer_of) {
  // encoder + one shared process block, >= 2 convs (no ReLU after the last), bias gradients from a ones row of
  // the augmented dW product (F_in, H < 32), node ids / message positions as u16; graphs of 65 .. 256 nodes one
  // per workgroup, 33 .. 64-node graphs (n_pad <= 128) in packs of 256 / n_pad
  const char* pk = getenv("GSC_GNN_LG_PACK");
  const bool big = NM > 64, packed = NM > (pk && pk[0] == '2' ? 0 : 32) && P <= 128 && gnn_lg_pack_enabled();
  if (!(Fin >= 1 && Fin <= 16 && H >= 1 && H <= 31 && (big || packed) && P >= NM && P <= kLgMaxNodes && M <= 8192 &&
        L >= 2 && L <= kClMaxLayers && n_blocks == 2))
    return false;
  for (int l = 0; l < L; ++l)
    if ((l == 0) != (layer_of[l] == 0)) return false;
  ClArgs a{};
  a.Fin = Fin; a.H = H; a.NM = NM; a.M = M; a.P = P; a.L = L; a.n_blocks = n_blocks;
  const int HV = lg_hv(H);
  if (packed && !big && lg_pack(a) < 2) return false;  // a pack of one small graph: the multi-tile kernels
  return lg_layout(a, HV, false).total <= 160 * 1024 && lg_layout(a, HV, true).total <= 160 * 1024;
}

template <int HV>
static void lg_launch_fwd(const ClArgs& a, hipStream_t st, int cus) {
  const LgLayout m = lg_layout(a, HV, false);
  const size_t lds = m.total;
  GSC_CHECK(lds <= 160 * 1024, "GNN (large-graph fused) forward working set exceeds LDS");
  const bool prof = lg_prof_on(), pk = m.G > 1;
  const void* fn = pk ? (prof ? (const void*)gnn_lg_fwd_kernel<HV, true, true> : (const void*)gnn_lg_fwd_kernel<HV, false, true>)
                      : (prof ? (const void*)gnn_lg_fwd_kernel<HV, true, false> : (const void*)gnn_lg_fwd_kernel<HV, false, false>);
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu > 2 ? 2 : (per_cu < 1 ? 1 : per_cu);
  long grid = (long)cus * per_cu;
  const long npk = (a.B + m.G - 1) / m.G;
  if (grid > npk) grid = npk;
  if (grid < 1) grid = 1;
  unsigned long long* pr = prof ? g_lg_prof : nullptr;
  hipLaunchKernelGGL(reinterpret_cast<void (*)(ClArgs, LgLayout, unsigned long long*)>(const_cast<void*>(fn)),
                     dim3((unsigned)grid), dim3(kLgThreads), lds, st, a, m, pr);
  check_launch();
}

template <int HV>
static int lg_launch_bwd(const ClArgs& a, hipStream_t st, int cus, int max_rows) {
  const LgLayout m = lg_layout(a, HV, true);
  const size_t lds = m.total;
  GSC_CHECK(lds <= 160 * 1024, "GNN (large-graph fused) backward working set exceeds LDS");
  const bool prof = lg_prof_on(), pk = m.G > 1;
  const char* e = getenv("GSC_LG_BWD_NL");
  const bool nl2 = e && e[0] == '2' && !pk;  // (A/B knob of the one-graph kernels)
  const void* fn = pk ? (prof ? (const void*)gnn_lg_bwd_kernel<HV, 4, true, true> : (const void*)gnn_lg_bwd_kernel<HV, 4, false, true>)
                 : nl2 ? (prof ? (const void*)gnn_lg_bwd_kernel<HV, 2, true, false> : (const void*)gnn_lg_bwd_kernel<HV, 2, false, false>)
                       : (prof ? (const void*)gnn_lg_bwd_kernel<HV, 4, true, false> : (const void*)gnn_lg_bwd_kernel<HV, 4, false, false>);
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long grid = cus;
  const long npk = (a.B + m.G - 1) / m.G;
  if (grid > npk) grid = npk;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  const dim3 blk(nl2 ? 512 : kLgBwdThreads);
  {  // a launch the device cannot run (LDS, threads x registers) must fail loudly, not leave the partials unwritten
    hipFuncAttributes fa{};
    GSC_HIP_CHECK(hipFuncGetAttributes(&fa, fn));
    int dev = 0, maxlds = 0;
    GSC_HIP_CHECK(hipGetDevice(&dev));
    GSC_HIP_CHECK(hipDeviceGetAttribute(&maxlds, hipDeviceAttributeSharedMemPerBlockOptin, dev));
    GSC_CHECK(fa.maxThreadsPerBlock >= (int)blk.x && (int)lds <= maxlds,
              "large-graph GNN backward: " + std::to_string(blk.x) + " threads / " + std::to_string(lds) +
                  " B LDS exceed the kernel's limits (" + std::to_string(fa.maxThreadsPerBlock) + " threads, " +
                  std::to_string(maxlds) + " B)");
  }
  unsigned long long* pr = prof ? g_lg_prof : nullptr;
  hipLaunchKernelGGL(reinterpret_cast<void (*)(ClArgs, LgLayout, unsigned long long*)>(const_cast<void*>(fn)),
                     dim3((unsigned)grid), blk, lds, st, a, m, pr);
  check_launch();
  return (int)grid;
}

static void lg_check(const ClArgs& a) {
  GSC_CHECK(a.P <= kLgMaxNodes && a.P >= a.NM && (long)lg_pack(a) * a.M <= 8192 && a.H <= 31 && a.Fin <= 16 &&
                a.L >= 2 && a.n_blocks == 2,
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
