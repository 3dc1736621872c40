// Layer-wise GATv2 for graphs too large for the fused per-graph kernels (e.g. the 200-node
// synthetic topologies of BASELINE config 5: a graph's working set exceeds one CU's LDS).
//
// One conv = three stages over the whole batch (rows = B graphs x P node slots):
//   node linears   [x_l | x_r] = h W^T + b          MFMA GEMM engine (csrc/ops/mlp.hip), K = Fi
//   attention      per target node: scores att . LeakyReLU(x_l[j] + x_r[i]) over its in-messages
//                  (CSR), PyG segment softmax, mean aggregation, bias, ReLU        (this file)
//   mean pool      per graph, fixed order                                        (this file)
// and the backward mirrors it: attention backward per target node (softmax / score / scatter
// terms; d x_r gathered per target, d x_l gathered per source through the source-sorted CSR -- no
// atomics), weight gradients dW = dX^T h and input gradients dX W on the GEMM engine, vector
// gradients by deterministic two-phase column sums.  Between convs the node linears of the next conv
// run in the attention kernel's epilogue and the input gradient dX W in the source gather's.
//
// Lanes: a 32-lane half-wave (H <= 32) or a whole wave (H <= 64) owns one (graph, node) with lane
// c = channel; message scores reduce over those lanes with xor shuffles.  Reference: PyG GATv2Conv as gatv2_dense_reference
// (gsc_amd/models/gnn.py) -- reference repo src/rlsp/agents/models.py:10-53.
#include <pybind11/pybind11.h>

#include "../common.h"
#include "gnn_mf.h"

namespace py = pybind11;

namespace gsc {

constexpr float kLwSlope = 0.2f;

// ---- MFMA node linears for the lane-per-node kernels (n_pad <= 256) ----------------------------------
// A graph's node rows as a bf16 [row][k] image (row stride kMfRS = 40: conflict-free 16-byte fragment
// reads), then one 32-row tile per wave and pass: X = rows W^T (+ b) on v_mfma_f32_32x32x16_bf16 with the
// H x H weights as fragments (K <= 32: two k-steps) -- instead of H^2 broadcast-LDS FMAs per lane.
// The image reuses a [P][HV] fp32 LDS region of the kernel: it needs ceil32(P) * 80 bytes.
__host__ __device__ constexpr bool lw_mfma_fits(int P, int HV) {
  return P <= 256 && HV >= 16 && ((P + 31) / 32) * 32 * kMfRS * 2 <= P * HV * 4;
}
// row i of the image from a lane's fp32 row (channels >= H and rows >= n are zero)
template <int HV>
__device__ __forceinline__ void lw_put_bf16_row(__bf16* img, int i, const float (&v)[HV], int H) {
  bf16x8 c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * q + j;
      c[q][j] = (__bf16)((k < HV && k < H) ? v[k < HV ? k : 0] : 0.f);
    }
#pragma unroll
  for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(img + i * kMfRS + 8 * q) = c[q];
}
// out[b*P + row][c] = sum_k img[row][k] Wa[c][k] (+ Wb-term) + bias for every row < P (lane column c < H).
// TRANS: the weights enter transposed (dX W: out[row][k] = sum_c img[row][c] W[c][k]).  imgb / wb optional
// (the second product accumulates into the same tile: dX_l W_l + dX_r W_r).
template <bool TRANS>
__device__ __forceinline__ void lw_mfma_rows(const __bf16* imga, const float* __restrict__ wa, const float* __restrict__ ba,
                                             float* __restrict__ outa, const __bf16* imgb, const float* __restrict__ wb,
                                             const float* __restrict__ bb, float* __restrict__ outb, int P, int H, long row0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  bf16x8 fa[2], fb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    fa[ks] = mf_wfrag(wa, H, H, r, 16 * ks + 8 * hh, TRANS);
    fb[ks] = wb ? mf_wfrag(wb, H, H, r, 16 * ks + 8 * hh, TRANS) : fa[ks];
  }
  const float bca = (ba && r < H) ? ba[r] : 0.f, bcb = (bb && r < H) ? bb[r] : 0.f;
  for (int t = wave; 32 * t < P; t += waves) {
    f32x16 xa, xb;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      xa[i] = bca;
      xb[i] = bcb;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(imga + (32 * t + r) * kMfRS + 16 * ks + 8 * hh);
      if (outb) {  // two outputs from one input image (x_l', x_r')
        xa = mf_mma(a, fa[ks], xa);
        xb = mf_mma(a, fb[ks], xb);
      } else {     // one output from two input images (dX_l W_l + dX_r W_r)
        const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(imgb + (32 * t + r) * kMfRS + 16 * ks + 8 * hh);
        xa = mf_mma(a, fa[ks], xa);
        xa = mf_mma(a2, fb[ks], xa);
      }
    }
    if (r < H) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = 32 * t + mf_row(i, hh);
        if (row < P) {
          outa[(row0 + row) * H + r] = xa[i];
          if (outb) outb[(row0 + row) * H + r] = xb[i];
        }
      }
    }
  }
}
constexpr int LW_U = 4;  // messages per group in the per-node loops (loads in flight together)

__device__ __forceinline__ void lw_stage_rows(const float* __restrict__ src, long r0, int nr, int w, float* dst);

struct LwGraph {
  const int32_t* topo;     // [B]
  const int32_t* nnodes;   // [T]
  const int32_t* in_ptr;   // [T, P+1]  messages into each node (target-sorted order)
  const int32_t* in_src;   // [T, M]    source of the q-th target-sorted message
  const int32_t* out_ptr;  // [T, P+1]  messages out of each node
  const int32_t* out_q;    // [T, M]    target-sorted position of the source-sorted messages
  const float* deg;        // [T, P]
  int B, P, M, H;
};

// sum over the NL lanes (32: half-wave, 64: wave) that own one node
template <int NL>
__device__ __forceinline__ float lw_sum(float v) {
#pragma unroll
  for (int o = NL / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, NL);
  return v;
}

__device__ __forceinline__ float leaky(float z) { return z > 0.f ? z : kLwSlope * z; }

// ---- forward attention + aggregation ---------------------------------------------------------------
// h_out[b,i,:] = act( sum_q alpha_q x_l[b,j_q,:] / deg_i + bias ),  alpha_q saved as [B, M]
// With nx.wl set, the epilogue also computes the next conv's node linears from the output row
// (x_l' = h W_l'^T + b_l', x_r' likewise; the H x H weights staged transposed in LDS, the row
// broadcast lane by lane), so the layer-to-layer GEMMs and the re-read of h_out disappear.
// first conv from a narrow input (Fi <= 8): x_l / x_r computed in the attention kernel (no node-linear pass)
struct LwFirst {
  const float* x;  // [B*P][Fi] (null: x_l / x_r come from memory)
  int Fi;
  const float* wl;  // [H][Fi]
  const float* bl;
  const float* wr;
  const float* br;
  float* xl_out;    // [B*P][H] (null: not needed -- no backward)
  float* xr_out;
};

struct LwNext {
  const float* wl;  // [H][H] (null: last conv)
  const float* bl;
  const float* wr;
  const float* br;
  float* xl;        // [B*P][H]
  float* xr;
};

template <int NL>
__global__ __launch_bounds__(256) void lw_attn_fwd_kernel(LwGraph g, const float* __restrict__ xl,
                                                          const float* __restrict__ xr, const float* __restrict__ att,
                                                          const float* __restrict__ bias, int relu,
                                                          float* __restrict__ h_out, float* __restrict__ alpha,
                                                          LwNext nx) {
  extern __shared__ float lw_wt[];  // [2][H][H]: W_l'^T, W_r'^T
  const int H = g.H;
  if (nx.wl) {
    for (int k = threadIdx.x; k < H * H; k += blockDim.x) {
      const int co = k / H, ci = k - co * H;  // W[co][ci] -> wt[ci][co]
      lw_wt[ci * H + co] = nx.wl[k];
      lw_wt[H * H + ci * H + co] = nx.wr[k];
    }
    __syncthreads();
  }
  const long node = (long)blockIdx.x * (256 / NL) + (threadIdx.x / NL);  // 256 / NL nodes per block
  const int c = threadIdx.x & (NL - 1);
  if (node >= (long)g.B * g.P) return;
  const int b = (int)(node / g.P), i = (int)(node - (long)b * g.P);
  const int t = g.topo[b];
  float* out = h_out + node * H;
  if (i >= g.nnodes[t]) {
    if (c < H) {
      out[c] = 0.f;
      if (nx.wl) {  // zero row: the node linears are the biases
        nx.xl[node * H + c] = nx.bl[c];
        nx.xr[node * H + c] = nx.br[c];
      }
    }
    return;
  }
  const int q0 = g.in_ptr[(long)t * (g.P + 1) + i], q1 = g.in_ptr[(long)t * (g.P + 1) + i + 1];
  const int32_t* src = g.in_src + (long)t * g.M;
  const float* xlb = xl + (long)b * g.P * H;
  const float xri = c < H ? xr[node * H + c] : 0.f;
  const float ac = c < H ? att[c] : 0.f;
  float* al = alpha + (long)b * g.M;
  // one pass over the in-messages with an online softmax (running max, rescaled sums); the raw
  // scores go to alpha (message q by lane (q - q0) mod NL) and are normalised afterwards
  // messages in groups of LW_U: the index and x_l row loads of a group are independent (in flight
  // together), then one rescale per group
  float mx = -__builtin_inff(), den = 0.f, acc = 0.f, s0 = 0.f, s1 = 0.f;
  for (int q = q0; q < q1; q += LW_U) {
    float xv[LW_U], sc[LW_U];
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      const int qq = q + u;
      xv[u] = (qq < q1 && c < H) ? xlb[(long)src[qq] * H + c] : 0.f;
    }
    float gm = mx;
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      sc[u] = lw_sum<NL>(ac * leaky(xv[u] + xri));
      if (q + u < q1) {
        if (c == ((q + u - q0) & (NL - 1))) {  // every lane holds the score (xor butterfly); raw scores
          const int k = (q + u - q0) / NL;     // stay in registers for the first 2 NL messages
          if (k == 0) s0 = sc[u];
          else if (k == 1) s1 = sc[u];
          else al[q + u] = sc[u];
        }
        gm = sc[u] > gm ? sc[u] : gm;
      }
    }
    if (gm > mx) {
      const float r = __expf(mx - gm);  // 0 on the first group (mx = -inf)
      den *= r;
      acc *= r;
      mx = gm;
    }
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      if (q + u < q1) {
        const float e = __expf(sc[u] - mx);
        den += e;
        acc += e * xv[u];
      }
    }
  }
  const float inv = 1.f / (den + 1e-16f);
  // each lane normalises the scores it holds (same-lane order for the rare ones kept in memory)
  for (int q = q0 + c, k = 0; q < q1; q += NL, ++k) al[q] = __expf((k == 0 ? s0 : k == 1 ? s1 : al[q]) - mx) * inv;
  float y = 0.f;
  if (c < H) {
    y = acc * inv / g.deg[(long)t * g.P + i] + bias[c];
    if (relu) y = y > 0.f ? y : 0.f;
    out[c] = y;
  }
  if (nx.wl) {
    float al_ = c < H ? nx.bl[c] : 0.f, ar_ = c < H ? nx.br[c] : 0.f;
    const int cc = c < H ? c : 0;
    for (int k = 0; k < H; ++k) {
      const float hk = __shfl(y, k, NL);
      al_ += lw_wt[k * H + cc] * hk;
      ar_ += lw_wt[H * H + k * H + cc] * hk;
    }
    if (c < H) {
      nx.xl[node * H + c] = al_;
      nx.xr[node * H + c] = ar_;
    }
  }
}

// Per-graph variant (the graph's x_l / x_r rows fit in LDS): one workgroup per graph stages its
// P x H x_l and x_r blocks with 16-byte loads, then 256 / NL lane groups take the nodes in turn and
// gather the message rows from LDS -- the HBM traffic is the coalesced block copies instead of one
// dependent row gather per message.  Same arithmetic as lw_attn_fwd_kernel.
template <int NL>
__global__ __launch_bounds__(256) void lw_graph_attn_fwd_kernel(LwGraph g, const float* __restrict__ xl,
                                                                const float* __restrict__ xr,
                                                                const float* __restrict__ att,
                                                                const float* __restrict__ bias, int relu,
                                                                float* __restrict__ h_out, float* __restrict__ alpha,
                                                                LwNext nx) {
  // LDS: x_l [P][H], x_r [P][H], W_l'^T, W_r'^T [H][H] (when nx.wl), in_ptr [P+1], in_src [M], deg [P]
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, PH = P * H;
  const int b = blockIdx.x;
  const int t = g.topo[b];
  float* s_xl = lw_g;
  float* s_xr = lw_g + PH;
  float* s_wt = lw_g + 2 * PH;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_wt + (nx.wl ? 2 * H * H : 0));
  int32_t* src = iptr + P + 1;
  float* s_deg = reinterpret_cast<float*>(src + g.M);
  lw_stage_rows(xl, (long)b * P, P, H, s_xl);
  lw_stage_rows(xr, (long)b * P, P, H, s_xr);
  if (nx.wl) {
    for (int k = threadIdx.x; k < H * H; k += blockDim.x) {
      const int co = k / H, ci = k - co * H;
      s_wt[ci * H + co] = nx.wl[k];
      s_wt[H * H + ci * H + co] = nx.wr[k];
    }
  }
  for (int k = threadIdx.x; k <= P; k += blockDim.x) iptr[k] = g.in_ptr[(long)t * (P + 1) + k];
  for (int k = threadIdx.x; k < g.M; k += blockDim.x) src[k] = g.in_src[(long)t * g.M + k];
  for (int k = threadIdx.x; k < P; k += blockDim.x) s_deg[k] = g.deg[(long)t * P + k];
  __syncthreads();
  const int n = g.nnodes[t];
  const int c = threadIdx.x & (NL - 1);
  const int cc = c < H ? c : 0;
  const float ac = c < H ? att[c] : 0.f;
  const float bc = c < H ? bias[c] : 0.f;
  float* al = alpha + (long)b * g.M;
  for (int i = threadIdx.x / NL; i < P; i += 256 / NL) {
    const long node = (long)b * P + i;
    if (i >= n) {
      if (c < H) {
        h_out[node * H + c] = 0.f;
        if (nx.wl) {
          nx.xl[node * H + c] = nx.bl[c];
          nx.xr[node * H + c] = nx.br[c];
        }
      }
      continue;
    }
    const int q0 = iptr[i], q1 = iptr[i + 1];
    const float xri = s_xr[i * H + cc];
    float mx = -__builtin_inff(), den = 0.f, acc = 0.f, s0 = 0.f, s1 = 0.f;
    for (int q = q0; q < q1; q += LW_U) {
      float xv[LW_U], sc[LW_U];
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        const int qq = q + u;
        xv[u] = (qq < q1 && c < H) ? s_xl[src[qq] * H + c] : 0.f;
      }
      float gm = mx;
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        sc[u] = lw_sum<NL>(ac * leaky(xv[u] + xri));
        if (q + u < q1) {
          if (c == ((q + u - q0) & (NL - 1))) {  // raw scores: registers for the first 2 NL messages
            const int k = (q + u - q0) / NL;
            if (k == 0) s0 = sc[u];
            else if (k == 1) s1 = sc[u];
            else al[q + u] = sc[u];
          }
          gm = sc[u] > gm ? sc[u] : gm;
        }
      }
      if (gm > mx) {
        const float r = __expf(mx - gm);
        den *= r;
        acc *= r;
        mx = gm;
      }
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        if (q + u < q1) {
          const float e = __expf(sc[u] - mx);
          den += e;
          acc += e * xv[u];
        }
      }
    }
    const float inv = 1.f / (den + 1e-16f);
    for (int q = q0 + c, k = 0; q < q1; q += NL, ++k) al[q] = __expf((k == 0 ? s0 : k == 1 ? s1 : al[q]) - mx) * inv;
    float y = 0.f;
    if (c < H) {
      y = acc * inv / s_deg[i] + bc;
      if (relu) y = y > 0.f ? y : 0.f;
      h_out[node * H + c] = y;
    }
    if (nx.wl) {
      float al_ = c < H ? nx.bl[c] : 0.f, ar_ = c < H ? nx.br[c] : 0.f;
      for (int k = 0; k < H; ++k) {
        const float hk = __shfl(y, k, NL);
        al_ += s_wt[k * H + cc] * hk;
        ar_ += s_wt[H * H + k * H + cc] * hk;
      }
      if (c < H) {
        nx.xl[node * H + c] = al_;
        nx.xr[node * H + c] = ar_;
      }
    }
  }
}

// A lane's H-float row from registers: 8-byte stores when the row is 8-byte aligned (fewer, wider
// store instructions than one per element), else element stores.
template <int HV>
__device__ __forceinline__ void lw_store_row(float* dst, const float (&v)[HV], int H) {
  if ((((uintptr_t)dst) & 7) == 0 && (H & 1) == 0) {
#pragma unroll
    for (int c = 0; c < HV; c += 2)
      if (c < H) *reinterpret_cast<float2*>(dst + c) = make_float2(v[c], v[c + 1]);
  } else {
#pragma unroll
    for (int c = 0; c < HV; ++c)
      if (c < H) dst[c] = v[c];
  }
}

// Lane-per-node forward (H <= 32): one workgroup per graph, one lane per target node.  The message
// scores are dot products over the lane's own registers (no cross-lane reductions, no shuffles); the
// graph's x_l rows sit in LDS with a padded row stride HV (16-byte reads), the raw scores in an LDS
// slot per message (each message has one target), and the next conv's node linears read W
// broadcast from LDS.  Same arithmetic as lw_attn_fwd_kernel.
template <int HV>
__global__ __launch_bounds__(256) void lw_lane_attn_fwd_kernel(LwGraph g, const float* __restrict__ xl,
                                                               const float* __restrict__ xr,
                                                               const float* __restrict__ att,
                                                               const float* __restrict__ bias, int relu,
                                                               float* __restrict__ h_out, float* __restrict__ alpha,
                                                               LwNext nx, float* __restrict__ emb) {
  // LDS: x_l [P][HV], W_l', W_r' [H][HV] (when nx.wl), raw scores [M], deg [P], in_ptr [P+1], in_src [M]
  // emb (last conv): the graph's mean pool, lane partial sums reduced in a fixed shuffle / wave order
  __shared__ float red[4][HV];
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, M = g.M;
  const int b = blockIdx.x, t = g.topo[b];
  float* s_xl = lw_g;
  float* s_w = s_xl + P * HV;
  float* s_sc = s_w + (nx.wl ? 2 * H * HV : 0);
  float* s_deg = s_sc + M;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_deg + P);
  int32_t* src = iptr + P + 1;
  const long base = (long)b * P * H;
  for (int k = threadIdx.x; k < P * HV; k += 256) {
    const int r = k / HV, c = k - r * HV;
    s_xl[k] = c < H ? xl[base + (long)r * H + c] : 0.f;
  }
  if (nx.wl) {
    for (int k = threadIdx.x; k < H * HV; k += 256) {
      const int r = k / HV, c = k - r * HV;
      s_w[k] = c < H ? nx.wl[r * H + c] : 0.f;
      s_w[H * HV + k] = c < H ? nx.wr[r * H + c] : 0.f;
    }
  }
  for (int k = threadIdx.x; k <= P; k += 256) {
    iptr[k] = g.in_ptr[(long)t * (P + 1) + k];
    if (k < P) s_deg[k] = g.deg[(long)t * P + k];
  }
  for (int k = threadIdx.x; k < M; k += 256) src[k] = g.in_src[(long)t * M + k];
  __syncthreads();
  float a_[HV], bi[HV];
#pragma unroll
  for (int c = 0; c < HV; ++c) {
    a_[c] = c < H ? att[c] : 0.f;
    bi[c] = c < H ? bias[c] : 0.f;
  }
  const int n = g.nnodes[t];
  float* al = alpha + (long)b * M;
  float ys[HV];
#pragma unroll
  for (int c = 0; c < HV; ++c) ys[c] = 0.f;
  for (int i = threadIdx.x; i < P; i += 256) {
    const long node = (long)b * P + i;
    float y[HV];
    if (i < n) {
      float xri[HV], acc[HV];
#pragma unroll
      for (int c = 0; c < HV; ++c) {
        xri[c] = c < H ? xr[node * H + c] : 0.f;
        acc[c] = 0.f;
      }
      const int q0 = iptr[i], q1 = iptr[i + 1];
      float mx = -__builtin_inff(), den = 0.f;
      for (int q = q0; q < q1; ++q) {
        const float4* row = reinterpret_cast<const float4*>(s_xl + src[q] * HV);
        float xj[HV];
#pragma unroll
        for (int v = 0; v < HV / 4; ++v) {
          const float4 f = row[v];
          xj[4 * v] = f.x;
          xj[4 * v + 1] = f.y;
          xj[4 * v + 2] = f.z;
          xj[4 * v + 3] = f.w;
        }
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < HV; ++c) s += a_[c] * leaky(xj[c] + xri[c]);
        s_sc[q] = s;
        if (s > mx) {
          const float r = __expf(mx - s);  // 0 for the first message
          den *= r;
#pragma unroll
          for (int c = 0; c < HV; ++c) acc[c] *= r;
          mx = s;
        }
        const float e = __expf(s - mx);
        den += e;
#pragma unroll
        for (int c = 0; c < HV; ++c) acc[c] += e * xj[c];
      }
      const float inv = 1.f / (den + 1e-16f);
      for (int q = q0; q < q1; ++q) al[q] = __expf(s_sc[q] - mx) * inv;
      const float sc = inv / s_deg[i];
#pragma unroll
      for (int c = 0; c < HV; ++c) {
        float v = acc[c] * sc + bi[c];
        if (relu) v = v > 0.f ? v : 0.f;
        y[c] = c < H ? v : 0.f;
        ys[c] += y[c];
      }
    } else {
#pragma unroll
      for (int c = 0; c < HV; ++c) y[c] = 0.f;
    }
    lw_store_row<HV>(h_out + node * H, y, H);
    if (nx.wl) {  // x_l'[co] = b_l'[co] + W_l'[co] . y  (W rows broadcast from LDS)
      float ol[HV], orr[HV];
#pragma unroll
      for (int co = 0; co < HV; ++co) {
        ol[co] = 0.f;
        orr[co] = 0.f;
        if (co < H) {
          const float4* wl4 = reinterpret_cast<const float4*>(s_w + co * HV);
          const float4* wr4 = reinterpret_cast<const float4*>(s_w + H * HV + co * HV);
          float sl = nx.bl[co], sr = nx.br[co];
#pragma unroll
          for (int v = 0; v < HV / 4; ++v) {
            const float4 fl = wl4[v], fr = wr4[v];
            sl += fl.x * y[4 * v] + fl.y * y[4 * v + 1] + fl.z * y[4 * v + 2] + fl.w * y[4 * v + 3];
            sr += fr.x * y[4 * v] + fr.y * y[4 * v + 1] + fr.z * y[4 * v + 2] + fr.w * y[4 * v + 3];
          }
          ol[co] = sl;
          orr[co] = sr;
        }
      }
      lw_store_row<HV>(nx.xl + node * H, ol, H);
      lw_store_row<HV>(nx.xr + node * H, orr, H);
    }
  }
  if (emb) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < HV; ++c) {
      float v = ys[c];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) red[w][c] = v;
    }
    __syncthreads();
    if ((int)threadIdx.x < H) {
      const int c = threadIdx.x;
      emb[(long)b * H + c] = ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) / (float)n;
    }
  }
}

template <int HV>
__device__ __forceinline__ void lw_load_row(float (&v)[HV], const float* src, int H);

// Staged lane-per-node forward (P <= 256, 16 <= H <= 32): one workgroup per graph, lane i = target node i.
// Latency-oriented: every global load of a graph is issued before the first LDS store (the x_l block as
// 16-B vectors, the lane's own x_r row, the topology rows: one HBM round trip per graph instead of one per
// staging-loop trip), only the gathered x_l rows live in LDS (row stride HV + 4 = 16 B x odd: the random
// row gathers spread over all bank quads), so ~32 KB per graph keeps 5 graphs in flight per CU.  The score
// a . LeakyReLU(z) runs as (1+s)/2 (a . z) + (1-s)/2 (a . |z|) -- two independent FMA chains with the |z|
// source modifier instead of a compare / select per channel.  Outputs leave through LDS with coalesced
// stores; the next conv's node linears run on the matrix cores (lw_mfma_rows).
template <int HV, bool FIRST = false>
__global__ __launch_bounds__(256, HV <= 24 ? 4 : 2) void lw_stage_attn_fwd_kernel(LwGraph g, const float* __restrict__ xl,
                                                                const float* __restrict__ xr,
                                                                const float* __restrict__ att,
                                                                const float* __restrict__ bias, int relu,
                                                                float* __restrict__ h_out, float* __restrict__ alpha,
                                                                LwNext nx, float* __restrict__ emb, LwFirst f0) {
  // LDS: x_l rows [P][RS] (then the output rows, then their bf16 image), scores [M] (then alpha), deg [P],
  //      in_ptr [P+1], in_src [M]
  constexpr int RS = HV + 4;
  constexpr int kV = 8;  // 16-B vectors per thread of the x_l block (P H <= 256 x 32)
  __shared__ float red[4][HV];
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, M = g.M;
  const int b = blockIdx.x, t = g.topo[b];
  float* s_xl = lw_g;
  float* s_sc = s_xl + P * RS;
  float* s_deg = s_sc + M;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_deg + P);
  int32_t* src = iptr + P + 1;
  const long base = (long)b * P * H;
  const int NE = P * H, i = threadIdx.x;
  const int n = g.nnodes[t];
  constexpr bool first = FIRST;  // f0.x set: x_l / x_r from the narrow input (own instantiation: registers)
  const bool vin = !first && (NE & 3) == 0 && ((reinterpret_cast<uintptr_t>(xl + base) & 15) == 0);
  const bool vec = (NE & 3) == 0 && (!h_out || (reinterpret_cast<uintptr_t>(h_out + base) & 15) == 0);
  // ---- all loads in flight together
  float4 v4[kV];
  float xin[8];  // first conv: the lane's input row
  if (first) {
#pragma unroll
    for (int k = 0; k < 8; ++k) xin[k] = (i < P && k < f0.Fi) ? f0.x[((long)b * P + i) * f0.Fi + k] : 0.f;
  } else if (vin) {
    const float4* x4 = reinterpret_cast<const float4*>(xl + base);
#pragma unroll
    for (int u = 0; u < kV; ++u) {
      const int j = i + 256 * u;
      if (j < NE / 4) v4[u] = x4[j];
    }
  }
  float xri[HV];
  if (!first && i < n) lw_load_row<HV>(xri, xr + base + (long)i * H, H);
  int ip = 0;
  float dg = 1.f;
  if (i <= P) ip = g.in_ptr[(long)t * (P + 1) + i];
  if (i < P) dg = g.deg[(long)t * P + i];
  int sv[kV];
#pragma unroll
  for (int u = 0; u < kV; ++u) {
    const int j = i + 256 * u;
    if (j < M) sv[u] = g.in_src[(long)t * M + j];
  }
  // ---- LDS images
  if (first) {  // x_l / x_r rows of node i from its input row (uniform weights: scalar loads)
    if (i < P) {
#pragma unroll
      for (int v = 0; v < HV / 4; ++v) {  // four channels at a time: x_l straight to LDS, x_r kept
        float xl4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * v + e;
          float al = 0.f, ar = 0.f;
          if (c < H) {
            al = f0.bl[c];
            ar = f0.br[c];
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (k < f0.Fi) {
                al = fmaf(f0.wl[c * f0.Fi + k], xin[k], al);
                ar = fmaf(f0.wr[c * f0.Fi + k], xin[k], ar);
              }
          }
          xl4[e] = al;
          xri[c] = ar;
        }
        reinterpret_cast<float4*>(s_xl + i * RS)[v] = make_float4(xl4[0], xl4[1], xl4[2], xl4[3]);
      }
    }
  } else if (vin) {
#pragma unroll
    for (int u = 0; u < kV; ++u) {
      const int j = i + 256 * u;
      if (j < NE / 4) {
        int r = (4 * j) / H, c = 4 * j - r * H;
        const float f[4] = {v4[u].x, v4[u].y, v4[u].z, v4[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s_xl[r * RS + c] = f[e];
          if (++c == H) { c = 0; ++r; }
        }
      }
    }
  } else {
    for (int k = i; k < NE; k += 256) {
      const int r = k / H, c = k - r * H;
      s_xl[r * RS + c] = xl[base + k];
    }
  }
  for (int k = first ? P * HV : i; k < P * (HV - H); k += 256) {  // padded channels are read: zero, not stale
    const int r = k / (HV - H), c = H + k - r * (HV - H);
    s_xl[r * RS + c] = 0.f;
  }
  if (i <= P) iptr[i] = ip;
  if (i < P) s_deg[i] = dg;
  if (P == 256 && i == 0) iptr[256] = g.in_ptr[(long)t * (P + 1) + 256];
#pragma unroll
  for (int u = 0; u < kV; ++u) {
    const int j = i + 256 * u;
    if (j < M) src[j] = sv[u];
  }
  for (int k = i + 256 * kV; k < M; k += 256) src[k] = g.in_src[(long)t * M + k];
  __syncthreads();
  if (first && f0.xl_out) {  // a backward reads x_l / x_r: coalesced stores (x_l from the LDS rows, x_r recomputed)
    for (int e0 = i; e0 < NE; e0 += 256) {
      const int r = e0 / H, c = e0 - r * H;
      float ar = f0.br[c];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        if (kk < f0.Fi) ar = fmaf(f0.wr[c * f0.Fi + kk], f0.x[((long)b * P + r) * f0.Fi + kk], ar);
      f0.xl_out[base + e0] = s_xl[r * RS + c];
      f0.xr_out[base + e0] = ar;
    }
  }
  // ---- lane = target node: scores, online softmax, aggregation
  float y[HV];
#pragma unroll
  for (int c = 0; c < HV; ++c) y[c] = 0.f;
  if (i < n) {
    float a_[HV], acc[HV];  // a_: uniform (scalar registers)
#pragma unroll
    for (int c = 0; c < HV; ++c) {
      a_[c] = c < H ? att[c] : 0.f;
      acc[c] = 0.f;
    }
    const int q0 = iptr[i], q1 = iptr[i + 1];
    float mx = -__builtin_inff(), den = 0.f;
    for (int q = q0; q < q1; ++q) {
      const float4* row = reinterpret_cast<const float4*>(s_xl + src[q] * RS);
      float xj[HV];
#pragma unroll
      for (int v = 0; v < HV / 4; ++v) {
        const float4 f = row[v];
        xj[4 * v] = f.x;
        xj[4 * v + 1] = f.y;
        xj[4 * v + 2] = f.z;
        xj[4 * v + 3] = f.w;
      }
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int c = 0; c < HV; ++c) {
        const float z = xj[c] + xri[c];
        s0 = fmaf(a_[c], z, s0);
        s1 = fmaf(a_[c], fabsf(z), s1);
      }
      const float sc = 0.5f * (1.f + kLwSlope) * s0 + 0.5f * (1.f - kLwSlope) * s1;
      s_sc[q] = sc;
      if (sc > mx) {
        const float r = __expf(mx - sc);  // 0 for the first message
        den *= r;
#pragma unroll
        for (int c = 0; c < HV; ++c) acc[c] *= r;
        mx = sc;
      }
      const float e = __expf(sc - mx);
      den += e;
#pragma unroll
      for (int c = 0; c < HV; ++c) acc[c] = fmaf(e, xj[c], acc[c]);
    }
    const float inv = 1.f / (den + 1e-16f);
    for (int q = q0; q < q1; ++q) s_sc[q] = __expf(s_sc[q] - mx) * inv;  // alpha, in place
    const float scl = inv / s_deg[i];
#pragma unroll
    for (int c = 0; c < HV; ++c) {
      float v = acc[c] * scl + (c < H ? bias[c] : 0.f);
      if (relu) v = v > 0.f ? v : 0.f;
      y[c] = c < H ? v : 0.f;
    }
  }
  __syncthreads();  // every lane is done gathering x_l rows: the output rows take their place
  if (h_out) {        // (null: a forward without a backward, or the last conv -- nobody reads the rows)
    if (i < P) {
      float4* ro = reinterpret_cast<float4*>(s_xl + i * RS);
#pragma unroll
      for (int v = 0; v < HV / 4; ++v) ro[v] = make_float4(y[4 * v], y[4 * v + 1], y[4 * v + 2], y[4 * v + 3]);
    }
    __syncthreads();
  }
  if (!h_out) {
  } else if (vec) {  // coalesced 16-B stores of the [P][H] block
    float4* o4 = reinterpret_cast<float4*>(h_out + base);
    for (int j = i; j < NE / 4; j += 256) {
      int r = (4 * j) / H, c = 4 * j - r * H;
      float f[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = s_xl[r * RS + c];
        if (++c == H) { c = 0; ++r; }
      }
      o4[j] = make_float4(f[0], f[1], f[2], f[3]);
    }
  } else {
    for (int k = i; k < NE; k += 256) {
      const int r = k / H, c = k - r * H;
      h_out[base + k] = s_xl[r * RS + c];
    }
  }
  if (alpha) {
    const int m = iptr[n];
    for (int q = i; q < m; q += 256) alpha[(long)b * M + q] = s_sc[q];
  }
  if (emb) {  // mean pool: lane partial sums reduced in a fixed shuffle / wave order
    const int lane = i & 63, w = i >> 6;
#pragma unroll
    for (int c = 0; c < HV; ++c) {
      float v = i < n ? y[c] : 0.f;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) red[w][c] = v;
    }
    __syncthreads();
    if (i < H) emb[(long)b * H + i] = ((red[0][i] + red[1][i]) + (red[2][i] + red[3][i])) / (float)n;
  }
  if (nx.wl) {  // the next conv's node linears on the matrix cores (after the pool: y dies in the bf16 image)
    __syncthreads();
    __bf16* s_y = reinterpret_cast<__bf16*>(s_xl);
    if (i < ((P + 31) & ~31)) lw_put_bf16_row<HV>(s_y, i, y, H);
    __syncthreads();
    lw_mfma_rows<false>(s_y, nx.wl, nx.bl, nx.xl, nullptr, nx.wr, nx.br, nx.xr, P, H, (long)b * P);
  }
}

// emb[b,:] = mean over the graph's real nodes of h[b,:,:]
template <int NL>
__global__ __launch_bounds__(256) void lw_pool_kernel(LwGraph g, const float* __restrict__ h, float* __restrict__ emb) {
  const long b = (long)blockIdx.x * (256 / NL) + (threadIdx.x / NL);
  const int c = threadIdx.x & (NL - 1);
  if (b >= g.B || c >= g.H) return;
  const int n = g.nnodes[g.topo[b]];
  const float* hb = h + b * g.P * g.H;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += hb[(long)i * g.H + c];
  emb[b * g.H + c] = s / (float)n;
}

// d h_last[b,i,:] = demb[b,:] / n for real nodes, 0 for padding
__global__ __launch_bounds__(256) void lw_pool_bwd_kernel(LwGraph g, const float* __restrict__ demb, float* __restrict__ dh) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)g.B * g.P * g.H;
  if (idx >= total) return;
  const long node = idx / g.H;
  const int c = (int)(idx - node * g.H);
  const int b = (int)(node / g.P), i = (int)(node - (long)b * g.P);
  const int n = g.nnodes[g.topo[b]];
  dh[idx] = i < n ? demb[(long)b * g.H + c] / (float)n : 0.f;
}

// ---- backward, per target node ---------------------------------------------------------------------
// In:  dh (gradient at this conv's output; overwritten by dY = dh * relu'(h_out)), h_out (null: no
//      ReLU), x_l, x_r, alpha.  Out: dxr[b,i,:] (gathered), per-message x_l gradients msg[b,q,:]
//      = alpha_q dY_i / deg_i + dz_q, per-node d att partials datt[b,i,:].
template <int NL>
__global__ __launch_bounds__(256) void lw_attn_bwd_kernel(LwGraph g, float* __restrict__ dh,
                                                          const float* __restrict__ h_out, const float* __restrict__ xl,
                                                          const float* __restrict__ xr,
                                                          const float* __restrict__ alpha, const float* __restrict__ att,
                                                          float* __restrict__ dxr, float* __restrict__ msg,
                                                          float* __restrict__ datt) {
  const long node = (long)blockIdx.x * (256 / NL) + (threadIdx.x / NL);
  const int c = threadIdx.x & (NL - 1);
  if (node >= (long)g.B * g.P) return;
  const int b = (int)(node / g.P), i = (int)(node - (long)b * g.P);
  const int t = g.topo[b];
  const int H = g.H;
  const bool ch = c < H;
  if (i >= g.nnodes[t]) {
    if (ch) {
      dh[node * H + c] = 0.f;
      dxr[node * H + c] = 0.f;
      datt[node * H + c] = 0.f;
    }
    return;
  }
  float dy = ch ? dh[node * H + c] : 0.f;
  if (h_out && ch && !(h_out[node * H + c] > 0.f)) dy = 0.f;
  if (ch) dh[node * H + c] = dy;
  const float gc = dy / g.deg[(long)t * g.P + i];
  const int q0 = g.in_ptr[(long)t * (g.P + 1) + i], q1 = g.in_ptr[(long)t * (g.P + 1) + i + 1];
  const int32_t* src = g.in_src + (long)t * g.M;
  const float* xlb = xl + (long)b * g.P * H;
  const float* al = alpha + (long)b * g.M;
  float* mb = msg + (long)b * g.M * H;
  const float xri = ch ? xr[node * H + c] : 0.f;
  const float ac = ch ? att[c] : 0.f;
  // sum_q' alpha_q' dalpha_q'  (groups of LW_U messages: loads in flight together)
  float sad = 0.f;
  for (int q = q0; q < q1; q += LW_U) {
    float xv[LW_U], a[LW_U];
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      const int qq = q + u;
      xv[u] = (qq < q1 && ch) ? xlb[(long)src[qq] * H + c] : 0.f;
      a[u] = qq < q1 ? al[qq] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < LW_U; ++u) sad += a[u] * lw_sum<NL>(gc * xv[u]);
  }
  float dxr_acc = 0.f, datt_acc = 0.f;
  for (int q = q0; q < q1; q += LW_U) {
    float xv[LW_U], a[LW_U];
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      const int qq = q + u;
      xv[u] = (qq < q1 && ch) ? xlb[(long)src[qq] * H + c] : 0.f;
      a[u] = qq < q1 ? al[qq] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < LW_U; ++u) {
      const float da = lw_sum<NL>(gc * xv[u]);
      const float de = a[u] * (da - sad);
      const float z = xv[u] + xri;
      const float dz = de * ac * (z > 0.f ? 1.f : kLwSlope);
      if (q + u < q1) {
        datt_acc += de * leaky(z);
        dxr_acc += dz;
        if (ch) mb[(long)(q + u) * H + c] = a[u] * gc + dz;
      }
    }
  }
  if (ch) {
    dxr[node * H + c] = dxr_acc;
    datt[node * H + c] = datt_acc;
  }
}

// dxl[b,j,:] = sum over messages out of j of msg[b,q,:]   (source-sorted CSR; no atomics).
// With wl set (a conv with an H-channel input), also the input gradient of the conv,
// dh[b,j,:] = dxl W_l + dxr W_r, from the row in registers (W read row-wise: lane = input channel).
template <int NL>
__global__ __launch_bounds__(256) void lw_src_gather_kernel(LwGraph g, const float* __restrict__ msg, float* __restrict__ dxl,
                                                            const float* __restrict__ dxr, const float* __restrict__ wl,
                                                            const float* __restrict__ wr, float* __restrict__ dh) {
  extern __shared__ float lw_w[];  // [2][H][H]: W_l, W_r (row = output channel)
  const int H = g.H;
  if (wl) {
    for (int k = threadIdx.x; k < H * H; k += blockDim.x) {
      lw_w[k] = wl[k];
      lw_w[H * H + k] = wr[k];
    }
    __syncthreads();
  }
  const long node = (long)blockIdx.x * (256 / NL) + (threadIdx.x / NL);
  const int c = threadIdx.x & (NL - 1);
  if (node >= (long)g.B * g.P) return;  // whole node groups exit together
  const int b = (int)(node / g.P), j = (int)(node - (long)b * g.P);
  const int t = g.topo[b];
  float s = 0.f;
  if (j < g.nnodes[t] && c < H) {
    const int p0 = g.out_ptr[(long)t * (g.P + 1) + j], p1 = g.out_ptr[(long)t * (g.P + 1) + j + 1];
    const int32_t* oq = g.out_q + (long)t * g.M;
    const float* mb = msg + (long)b * g.M * H;
    for (int p = p0; p < p1; p += LW_U) {
      float v[LW_U];
#pragma unroll
      for (int u = 0; u < LW_U; ++u) v[u] = p + u < p1 ? mb[(long)oq[p + u] * H + c] : 0.f;
#pragma unroll
      for (int u = 0; u < LW_U; ++u) s += v[u];
    }
  }
  if (c < H) dxl[node * H + c] = s;
  if (wl) {
    const float r = c < H ? dxr[node * H + c] : 0.f;
    const int cc = c < H ? c : 0;
    float d = 0.f;
    for (int k = 0; k < H; ++k) {
      const float lk = __shfl(s, k, NL), rk = __shfl(r, k, NL);
      d += lk * lw_w[k * H + cc] + rk * lw_w[H * H + k * H + cc];
    }
    if (c < H) dh[node * H + c] = d;
  }
}

// dh[r, :] *= (h[r, :] > 0)  (ReLU of the layer below; h = that layer's output)
__global__ __launch_bounds__(256) void lw_relu_mask_kernel(float* dh, const float* h, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !(h[i] > 0.f)) dh[i] = 0.f;
}

// Per-graph backward (x_l block in LDS): phase 1 = lw_attn_bwd_kernel per target node with the
// message rows read from LDS; workgroup barrier (the block's global msg / dxr stores are visible to
// it); phase 2 = lw_src_gather_kernel per source node (+ the input gradient, W_l, W_r in LDS).
template <int NL>
__global__ __launch_bounds__(256) void lw_graph_attn_bwd_kernel(LwGraph g, float* __restrict__ dh,
                                                                const float* __restrict__ h_out,
                                                                const float* __restrict__ xl,
                                                                const float* __restrict__ xr,
                                                                const float* __restrict__ alpha,
                                                                const float* __restrict__ att, float* __restrict__ dxr,
                                                                float* __restrict__ msg, float* __restrict__ datt,
                                                                float* __restrict__ dxl, const float* __restrict__ wl,
                                                                const float* __restrict__ wr, float* __restrict__ dh_in) {
  // LDS: x_l [P][H], (W_l, W_r [H][H]), alpha [M], deg [P], in_ptr / out_ptr [P+1], in_src / out_q [M]
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, PH = P * H, M = g.M;
  const int b = blockIdx.x;
  const int t = g.topo[b];
  float* s_xl = lw_g;
  float* s_w = lw_g + PH;
  float* al = s_w + (wl ? 2 * H * H : 0);
  float* s_deg = al + M;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_deg + P);
  int32_t* optr = iptr + P + 1;
  int32_t* src = optr + P + 1;
  int32_t* oq = src + M;
  lw_stage_rows(xl, (long)b * P, P, H, s_xl);
  if (wl) {
    for (int k = threadIdx.x; k < H * H; k += blockDim.x) {
      s_w[k] = wl[k];
      s_w[H * H + k] = wr[k];
    }
  }
  for (int k = threadIdx.x; k < M; k += blockDim.x) {
    al[k] = alpha[(long)b * M + k];
    src[k] = g.in_src[(long)t * M + k];
    oq[k] = g.out_q[(long)t * M + k];
  }
  for (int k = threadIdx.x; k <= P; k += blockDim.x) {
    iptr[k] = g.in_ptr[(long)t * (P + 1) + k];
    optr[k] = g.out_ptr[(long)t * (P + 1) + k];
    if (k < P) s_deg[k] = g.deg[(long)t * P + k];
  }
  __syncthreads();
  const int n = g.nnodes[t];
  const int c = threadIdx.x & (NL - 1);
  const bool ch = c < H;
  const int cc = ch ? c : 0;
  const float ac = ch ? att[c] : 0.f;
  float* mb = msg + (long)b * g.M * H;
  for (int i = threadIdx.x / NL; i < P; i += 256 / NL) {
    const long node = (long)b * P + i;
    if (i >= n) {
      if (ch) {
        dh[node * H + c] = 0.f;
        dxr[node * H + c] = 0.f;
        datt[node * H + c] = 0.f;
      }
      continue;
    }
    float dy = ch ? dh[node * H + c] : 0.f;
    if (h_out && ch && !(h_out[node * H + c] > 0.f)) dy = 0.f;
    if (ch) dh[node * H + c] = dy;
    const float gc = dy / s_deg[i];
    const int q0 = iptr[i], q1 = iptr[i + 1];
    const float xri = ch ? xr[node * H + c] : 0.f;
    float sad = 0.f;
    for (int q = q0; q < q1; q += LW_U) {
      float xv[LW_U], a[LW_U];
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        const int qq = q + u;
        xv[u] = (qq < q1 && ch) ? s_xl[src[qq] * H + c] : 0.f;
        a[u] = qq < q1 ? al[qq] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < LW_U; ++u) sad += a[u] * lw_sum<NL>(gc * xv[u]);
    }
    float dxr_acc = 0.f, datt_acc = 0.f;
    for (int q = q0; q < q1; q += LW_U) {
      float xv[LW_U], a[LW_U];
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        const int qq = q + u;
        xv[u] = (qq < q1 && ch) ? s_xl[src[qq] * H + c] : 0.f;
        a[u] = qq < q1 ? al[qq] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < LW_U; ++u) {
        const float da = lw_sum<NL>(gc * xv[u]);
        const float de = a[u] * (da - sad);
        const float z = xv[u] + xri;
        const float dz = de * ac * (z > 0.f ? 1.f : kLwSlope);
        if (q + u < q1) {
          datt_acc += de * leaky(z);
          dxr_acc += dz;
          if (ch) mb[(long)(q + u) * H + c] = a[u] * gc + dz;
        }
      }
    }
    if (ch) {
      dxr[node * H + c] = dxr_acc;
      datt[node * H + c] = datt_acc;
    }
  }
  __syncthreads();  // msg / dxr of this graph complete
  for (int j = threadIdx.x / NL; j < P; j += 256 / NL) {
    const long node = (long)b * P + j;
    float sum = 0.f;
    if (j < n && ch) {
      const int p0 = optr[j], p1 = optr[j + 1];
      for (int p = p0; p < p1; p += LW_U) {
        float v[LW_U];
#pragma unroll
        for (int u = 0; u < LW_U; ++u) v[u] = p + u < p1 ? mb[(long)oq[p + u] * H + c] : 0.f;
#pragma unroll
        for (int u = 0; u < LW_U; ++u) sum += v[u];
      }
    }
    if (ch) dxl[node * H + c] = sum;
    if (wl) {
      const float r = ch ? dxr[node * H + c] : 0.f;
      float d = 0.f;
      for (int k = 0; k < H; ++k) {
        const float lk = __shfl(sum, k, NL), rk = __shfl(r, k, NL);
        d += lk * s_w[k * H + cc] + rk * s_w[H * H + k * H + cc];
      }
      if (ch) dh_in[node * H + c] = d;
    }
  }
}

template <int HV>
__device__ __forceinline__ void lw_load_row(float (&v)[HV], const float* src, int H) {
  if ((((uintptr_t)src) & 7) == 0 && (H & 1) == 0) {
#pragma unroll
    for (int c = 0; c < HV; c += 2) {
      if (c < H) {
        const float2 f = *reinterpret_cast<const float2*>(src + c);
        v[c] = f.x;
        v[c + 1] = f.y;
      } else {
        v[c] = 0.f;
        v[c + 1] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < HV; ++c) v[c] = c < H ? src[c] : 0.f;
  }
}

// Lane-per-node backward (H <= 32), one workgroup per graph, no per-message rows in memory:
// phase 1, lane = target node i -- dY (ReLU gate), g_i = dY / deg_i, the softmax / score terms
// over its in-messages (x_l rows from LDS): d x_r, d att rows, and per message q the scalar
// de_q = alpha_q (da_q - sum alpha da) and its target (LDS), g_i rows (LDS); barrier; x_r rows
// replace x_l in LDS; phase 2, lane = source node j -- d x_l[j] = sum over its out-messages (fixed
// source-sorted order) of alpha_q g_i + de_q att * LeakyReLU'(x_l[j] + x_r[i]), recomputed from
// LDS, and with wl the input gradient d x_l W_l + d x_r W_r (W rows broadcast from LDS).  Same
// arithmetic as lw_attn_bwd_kernel + lw_src_gather_kernel.
template <int HV, bool MF = false>
__global__ __launch_bounds__(256) void lw_lane_attn_bwd_kernel(LwGraph g, float* __restrict__ dh,
                                                               const float* __restrict__ h_out,
                                                               const float* __restrict__ xl,
                                                               const float* __restrict__ xr,
                                                               const float* __restrict__ alpha,
                                                               const float* __restrict__ att, float* __restrict__ dxr,
                                                               float* __restrict__ datt, float* __restrict__ dxl,
                                                               const float* __restrict__ wl,
                                                               const float* __restrict__ wr, float* __restrict__ dh_in) {
  // LDS: rows [P][HV] (x_l, then x_r), g [P][HV], (W_l, W_r [H][HV]), alpha, de [M], deg [P],
  //      in_ptr / out_ptr [P+1], in_src / out_q / target [M]
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, M = g.M;
  const int b = blockIdx.x, t = g.topo[b];
  float* s_rows = lw_g;
  float* s_g = s_rows + P * HV;
  float* s_w = s_g + P * HV;
  float* al = s_w + (wl && !MF ? 2 * H * HV : 0);  // MF: no staged W (fragments from L2)
  float* s_de = al + M;
  float* s_deg = s_de + M;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_deg + P);
  int32_t* optr = iptr + P + 1;
  int32_t* src = optr + P + 1;
  int32_t* oq = src + M;
  int32_t* tgt = oq + M;
  const long base = (long)b * P * H;
  for (int k = threadIdx.x; k < P * HV; k += 256) {
    const int r = k / HV, c = k - r * HV;
    s_rows[k] = c < H ? xl[base + (long)r * H + c] : 0.f;
    s_g[k] = 0.f;
  }
  if (wl && !MF) {
    for (int k = threadIdx.x; k < H * HV; k += 256) {
      const int r = k / HV, c = k - r * HV;
      s_w[k] = c < H ? wl[r * H + c] : 0.f;
      s_w[H * HV + k] = c < H ? wr[r * H + c] : 0.f;
    }
  }
  for (int k = threadIdx.x; k < M; k += 256) {
    al[k] = alpha[(long)b * M + k];
    src[k] = g.in_src[(long)t * M + k];
    oq[k] = g.out_q[(long)t * M + k];
    s_de[k] = 0.f;
    tgt[k] = 0;
  }
  for (int k = threadIdx.x; k <= P; k += 256) {
    iptr[k] = g.in_ptr[(long)t * (P + 1) + k];
    optr[k] = g.out_ptr[(long)t * (P + 1) + k];
    if (k < P) s_deg[k] = g.deg[(long)t * P + k];
  }
  __syncthreads();
  float a_[HV];
#pragma unroll
  for (int c = 0; c < HV; ++c) a_[c] = c < H ? att[c] : 0.f;
  const int n = g.nnodes[t];
  for (int i = threadIdx.x; i < P; i += 256) {
    const long node = (long)b * P + i;
    float d1[HV], d2[HV];  // d x_r, d att
#pragma unroll
    for (int c = 0; c < HV; ++c) {
      d1[c] = 0.f;
      d2[c] = 0.f;
    }
    if (i < n) {
      float gc[HV], xri[HV];
      lw_load_row<HV>(gc, dh + node * H, H);
      if (h_out) {
        float ho[HV];
        lw_load_row<HV>(ho, h_out + node * H, H);
#pragma unroll
        for (int c = 0; c < HV; ++c) gc[c] = ho[c] > 0.f ? gc[c] : 0.f;
      }
      lw_store_row<HV>(dh + node * H, gc, H);  // dY (the bias gradient's rows)
      const float inv_deg = 1.f / s_deg[i];
#pragma unroll
      for (int c = 0; c < HV; ++c) {
        gc[c] *= inv_deg;
        s_g[i * HV + c] = gc[c];
      }
      lw_load_row<HV>(xri, xr + node * H, H);
      const int q0 = iptr[i], q1 = iptr[i + 1];
      float sad = 0.f;
      for (int q = q0; q < q1; ++q) {
        const float4* row = reinterpret_cast<const float4*>(s_rows + src[q] * HV);
        float da = 0.f;
#pragma unroll
        for (int v = 0; v < HV / 4; ++v) {
          const float4 f = row[v];
          da += gc[4 * v] * f.x + gc[4 * v + 1] * f.y + gc[4 * v + 2] * f.z + gc[4 * v + 3] * f.w;
        }
        sad += al[q] * da;
      }
      for (int q = q0; q < q1; ++q) {
        const float4* row = reinterpret_cast<const float4*>(s_rows + src[q] * HV);
        float xj[HV];
#pragma unroll
        for (int v = 0; v < HV / 4; ++v) {
          const float4 f = row[v];
          xj[4 * v] = f.x;
          xj[4 * v + 1] = f.y;
          xj[4 * v + 2] = f.z;
          xj[4 * v + 3] = f.w;
        }
        float da = 0.f;
#pragma unroll
        for (int c = 0; c < HV; ++c) da += gc[c] * xj[c];
        const float de = al[q] * (da - sad);
        s_de[q] = de;
        tgt[q] = i;
#pragma unroll
        for (int c = 0; c < HV; ++c) {
          const float z = xj[c] + xri[c];
          d2[c] += de * leaky(z);
          d1[c] += de * a_[c] * (z > 0.f ? 1.f : kLwSlope);
        }
      }
    } else {
      float z[HV];
#pragma unroll
      for (int c = 0; c < HV; ++c) z[c] = 0.f;
      lw_store_row<HV>(dh + node * H, z, H);
    }
    lw_store_row<HV>(dxr + node * H, d1, H);
    lw_store_row<HV>(datt + node * H, d2, H);
  }
  __syncthreads();  // phase 1 done with x_l in LDS; g / de / targets complete
  for (int k = threadIdx.x; k < P * HV; k += 256) {
    const int r = k / HV, c = k - r * HV;
    s_rows[k] = c < H ? xr[base + (long)r * H + c] : 0.f;
  }
  __syncthreads();
  float skeep[HV], rkeep[HV];  // MF: this thread's (only) source row of d x_l / d x_r for the MFMA epilogue
#pragma unroll
  for (int c = 0; c < HV; ++c) skeep[c] = rkeep[c] = 0.f;
  for (int j = threadIdx.x; j < P; j += 256) {
    const long node = (long)b * P + j;
    float s[HV];
#pragma unroll
    for (int c = 0; c < HV; ++c) s[c] = 0.f;
    if (j < n) {
      float xlj[HV];
      lw_load_row<HV>(xlj, xl + node * H, H);
      const int p0 = optr[j], p1 = optr[j + 1];
      for (int p = p0; p < p1; ++p) {
        const int q = oq[p];
        const int i = tgt[q];
        const float aq = al[q], de = s_de[q];
        const float4* xr4 = reinterpret_cast<const float4*>(s_rows + i * HV);
        const float4* g4 = reinterpret_cast<const float4*>(s_g + i * HV);
#pragma unroll
        for (int v = 0; v < HV / 4; ++v) {
          const float4 fr = xr4[v], fg = g4[v];
          const float zr[4] = {fr.x, fr.y, fr.z, fr.w}, gg[4] = {fg.x, fg.y, fg.z, fg.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = 4 * v + e;
            const float z = xlj[c] + zr[e];
            s[c] += aq * gg[e] + de * a_[c] * (z > 0.f ? 1.f : kLwSlope);
          }
        }
      }
    }
    lw_store_row<HV>(dxl + node * H, s, H);
    if constexpr (MF) {
      if (wl) {
        lw_load_row<HV>(rkeep, dxr + node * H, H);  // written by this lane in phase 1 (same node)
#pragma unroll
        for (int c = 0; c < HV; ++c) skeep[c] = s[c];
      }
    } else if (wl) {
      float r[HV], d[HV];
      lw_load_row<HV>(r, dxr + node * H, H);  // written by this lane in phase 1 (same node)
#pragma unroll
      for (int c = 0; c < HV; ++c) d[c] = 0.f;
#pragma unroll
      for (int co = 0; co < HV; ++co) {
        if (co < H) {
          const float4* wl4 = reinterpret_cast<const float4*>(s_w + co * HV);
          const float4* wr4 = reinterpret_cast<const float4*>(s_w + H * HV + co * HV);
#pragma unroll
          for (int v = 0; v < HV / 4; ++v) {
            const float4 fl = wl4[v], fr = wr4[v];
            d[4 * v] += s[co] * fl.x + r[co] * fr.x;
            d[4 * v + 1] += s[co] * fl.y + r[co] * fr.y;
            d[4 * v + 2] += s[co] * fl.z + r[co] * fr.z;
            d[4 * v + 3] += s[co] * fl.w + r[co] * fr.w;
          }
        }
      }
      lw_store_row<HV>(dh_in + node * H, d, H);
    }
  }
  if constexpr (MF) {
    if (wl) {  // input gradient d x_l W_l + d x_r W_r on the matrix cores
      __syncthreads();  // phase 2 is done with the x_r / g rows: the bf16 images reuse their LDS
      __bf16* img_l = reinterpret_cast<__bf16*>(s_rows);
      __bf16* img_r = reinterpret_cast<__bf16*>(s_g);
      if ((int)threadIdx.x < ((P + 31) & ~31)) {
        lw_put_bf16_row<HV>(img_l, threadIdx.x, skeep, H);
        lw_put_bf16_row<HV>(img_r, threadIdx.x, rkeep, H);
      }
      __syncthreads();
      lw_mfma_rows<true>(img_l, wl, nullptr, dh_in, img_r, wr, nullptr, nullptr, P, H, (long)b * P);
    }
  }
}

// [P][H] block <-> LDS rows [P][LD] (channels >= H untouched), 16-B global vectors (caller checks alignment)
template <int LD, int KV>
__device__ __forceinline__ void lw_block_load(float4 (&v)[KV], const float* src, int NE) {
  const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int j = threadIdx.x + 256 * u;
    if (j < NE / 4) v[u] = s4[j];
  }
}
template <int LD, int KV>
__device__ __forceinline__ void lw_block_to_lds(const float4 (&v)[KV], float* rows, int NE, int H) {
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int j = threadIdx.x + 256 * u;
    if (j < NE / 4) {
      int r = (4 * j) / H, c = 4 * j - r * H;
      const float f[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rows[r * LD + c] = f[e];
        if (++c == H) { c = 0; ++r; }
      }
    }
  }
}
template <int LD>
__device__ __forceinline__ void lw_lds_to_block(float* dst, const float* rows, int NE, int H) {
  float4* d4 = reinterpret_cast<float4*>(dst);
  for (int j = threadIdx.x; j < NE / 4; j += 256) {
    int r = (4 * j) / H, c = 4 * j - r * H;
    float f[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[e] = rows[r * LD + c];
      if (++c == H) { c = 0; ++r; }
    }
    d4[j] = make_float4(f[0], f[1], f[2], f[3]);
  }
}
template <int HV>
__device__ __forceinline__ void lw_put_row(float* rows, int i, const float (&v)[HV]) {
  float4* o = reinterpret_cast<float4*>(rows + i * HV);
#pragma unroll
  for (int k = 0; k < HV / 4; ++k) o[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}
template <int HV>
__device__ __forceinline__ void lw_get_row(float (&v)[HV], const float* rows, int i) {
  const float4* o = reinterpret_cast<const float4*>(rows + i * HV);
#pragma unroll
  for (int k = 0; k < HV / 4; ++k) {
    const float4 f = o[k];
    v[4 * k] = f.x;
    v[4 * k + 1] = f.y;
    v[4 * k + 2] = f.z;
    v[4 * k + 3] = f.w;
  }
}

// Staged lane-per-node backward (P <= 256, 16 <= H <= 32, 16-B aligned [P][H] blocks): the arithmetic of
// lw_lane_attn_bwd_kernel, laid out for latency and occupancy.  Every global load of a graph is issued
// before the first LDS store (x_l, dh, h_out blocks as 16-B vectors, alpha, the topology rows, the lane's
// own x_r / x_l rows); two [P][HV] row images (x_l then x_r; g) plus byte / short message indices keep a
// 200-node graph at ~53 KB (3 graphs per CU); the gated dY goes back to dh from the staging registers;
// phase 1 (lane = target node) and phase 2 (lane = source node) read only LDS; x_r replaces x_l in LDS
// between them (L2-hot reload).  d x_l / d x_r / d att leave through LDS with coalesced 16-B stores, and
// the input gradient d x_l W_l + d x_r W_r runs on the matrix cores (lw_mfma_rows).
template <int HV>
__global__ __launch_bounds__(256, HV <= 24 ? 3 : 2) void lw_stage_attn_bwd_kernel(LwGraph g, float* __restrict__ dh,
                                                                   const float* __restrict__ h_out,
                                                                   const float* __restrict__ xl,
                                                                   const float* __restrict__ xr,
                                                                   const float* __restrict__ alpha,
                                                                   const float* __restrict__ att, float* __restrict__ dxr,
                                                                   float* __restrict__ datt, float* __restrict__ dxl,
                                                                   const float* __restrict__ wl,
                                                                   const float* __restrict__ wr, float* __restrict__ dh_in,
                                                                   float* __restrict__ vpart,
                                                                   const float* __restrict__ demb) {
  // demb (optional, [B][H]): the last conv's incoming gradient is the mean-pool backward, formed here
  // (demb / n on the real nodes) instead of read from dh (no separate pool-backward pass)
  // vpart (optional, [B][H]): the graph's d att row sum instead of the d att rows (lw_conv_grads_v)
  // LDS: rows [P][HV] (x_l, then x_r, then outputs), g [P][HV], alpha, de [M] (fp32), deg [P], in_ptr / out_ptr
  //      [P+1], out_q [M] (u16), in_src / target [M] (u8)
  constexpr int KV = HV / 4;  // 16-B vectors per thread of a [P][H] block (P H <= 256 HV)
  extern __shared__ __attribute__((aligned(16))) float lw_g[];
  const int H = g.H, P = g.P, M = g.M;
  const int b = blockIdx.x, t = g.topo[b];
  float* s_rows = lw_g;
  float* s_g = s_rows + P * HV;
  float* al = s_g + P * HV;
  float* s_de = al + M;
  float* s_deg = s_de + M;
  int32_t* iptr = reinterpret_cast<int32_t*>(s_deg + P);
  int32_t* optr = iptr + P + 1;
  uint16_t* oq = reinterpret_cast<uint16_t*>(optr + P + 1);
  uint8_t* src = reinterpret_cast<uint8_t*>(oq + M);
  uint8_t* tgt = src + M;
  const long base = (long)b * P * H;
  const int NE = P * H, i = threadIdx.x;
  const int n = g.nnodes[t];
  // ---- every load in flight together
  float4 vx[KV], vd[KV], vh[KV];
  lw_block_load<HV, KV>(vx, xl + base, NE);
  if (demb) {
    const float inv_n = 1.f / (float)n;
#pragma unroll
    for (int u = 0; u < KV; ++u) {
      const int j = i + 256 * u;
      if (j < NE / 4) {
        int c = (4 * j) % H;
        float f[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[e] = demb[(long)b * H + c] * inv_n;  // rows >= n are zeroed below with the gate
          if (++c == H) c = 0;
        }
        vd[u] = make_float4(f[0], f[1], f[2], f[3]);
      }
    }
  } else {
    lw_block_load<HV, KV>(vd, dh + base, NE);
  }
  if (h_out) lw_block_load<HV, KV>(vh, h_out + base, NE);
  float xri[HV];
  if (i < n) lw_load_row<HV>(xri, xr + base + (long)i * H, H);
  int ip = 0, op = 0;
  float dg = 1.f;
  if (i <= P) {
    ip = g.in_ptr[(long)t * (P + 1) + i];
    op = g.out_ptr[(long)t * (P + 1) + i];
  }
  if (i < P) dg = g.deg[(long)t * P + i];
  for (int k = i; k < M; k += 256) {
    al[k] = alpha[(long)b * M + k];
    src[k] = (uint8_t)g.in_src[(long)t * M + k];
    oq[k] = (uint16_t)g.out_q[(long)t * M + k];
  }
  // ---- LDS images; dY = dh (ReLU-gated by the conv output, padded nodes 0) back to dh
  lw_block_to_lds<HV, KV>(vx, s_rows, NE, H);
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int j = i + 256 * u;
    if (j < NE / 4) {
      float f[4] = {vd[u].x, vd[u].y, vd[u].z, vd[u].w};
      if (h_out) {
        const float o[4] = {vh[u].x, vh[u].y, vh[u].z, vh[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = o[e] > 0.f ? f[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((4 * j + e) / H >= n) f[e] = 0.f;
      vd[u] = make_float4(f[0], f[1], f[2], f[3]);
      reinterpret_cast<float4*>(dh + base)[j] = vd[u];
    }
  }
  lw_block_to_lds<HV, KV>(vd, s_g, NE, H);
  for (int k = i; k < P * (HV - H); k += 256) {  // padded channels: read by the row loads, must be finite
    const int r = k / (HV - H), c = H + k - r * (HV - H);
    s_rows[r * HV + c] = 0.f;
    s_g[r * HV + c] = 0.f;
  }
  if (i <= P) {
    iptr[i] = ip;
    optr[i] = op;
  }
  if (i < P) s_deg[i] = dg;
  if (P == 256 && i == 0) {
    iptr[256] = g.in_ptr[(long)t * (P + 1) + 256];
    optr[256] = g.out_ptr[(long)t * (P + 1) + 256];
  }
  __syncthreads();
  float a_[HV];
#pragma unroll
  for (int c = 0; c < HV; ++c) a_[c] = c < H ? att[c] : 0.f;
  // ---- phase 1: lane = target node
  float d1[HV], d2[HV];  // d x_r, d att
#pragma unroll
  for (int c = 0; c < HV; ++c) {
    d1[c] = 0.f;
    d2[c] = 0.f;
  }
  if (i < n) {
    float gc[HV];
    lw_get_row<HV>(gc, s_g, i);
    const float inv_deg = 1.f / s_deg[i];
#pragma unroll
    for (int c = 0; c < HV; ++c) gc[c] *= inv_deg;
    lw_put_row<HV>(s_g, i, gc);  // own row: phase 2 reads the scaled rows after the barrier
    const int q0 = iptr[i], q1 = iptr[i + 1];
    float sad = 0.f;
    for (int q = q0; q < q1; ++q) {
      const float4* row = reinterpret_cast<const float4*>(s_rows + src[q] * HV);
      float da = 0.f;
#pragma unroll
      for (int v = 0; v < HV / 4; ++v) {
        const float4 f = row[v];
        da += gc[4 * v] * f.x + gc[4 * v + 1] * f.y + gc[4 * v + 2] * f.z + gc[4 * v + 3] * f.w;
      }
      sad += al[q] * da;
    }
    for (int q = q0; q < q1; ++q) {
      float xj[HV];
      lw_get_row<HV>(xj, s_rows, src[q]);
      float da = 0.f;
#pragma unroll
      for (int c = 0; c < HV; ++c) da += gc[c] * xj[c];
      const float de = al[q] * (da - sad);
      s_de[q] = de;
      tgt[q] = (uint8_t)i;
#pragma unroll
      for (int c = 0; c < HV; ++c) {
        const float z = xj[c] + xri[c];
        d2[c] += de * leaky(z);
        d1[c] += de * a_[c] * (z > 0.f ? 1.f : kLwSlope);
      }
    }
  }
  float xlj[HV];  // the lane's own x_l row for phase 2, before x_r replaces the image
  if (i < n) lw_get_row<HV>(xlj, s_rows, i);
  __syncthreads();  // phase 1 is done with the x_l rows; scaled g, de and targets complete
  {
    float4 vr[KV];  // x_r block (L2-hot: the lanes' own-row reads above)
    lw_block_load<HV, KV>(vr, xr + base, NE);
    lw_block_to_lds<HV, KV>(vr, s_rows, NE, H);
  }
  __syncthreads();
  // ---- phase 2: lane = source node
  float s[HV];  // d x_l
#pragma unroll
  for (int c = 0; c < HV; ++c) s[c] = 0.f;
  if (i < n) {
    const int p0 = optr[i], p1 = optr[i + 1];
    for (int p = p0; p < p1; ++p) {
      const int q = oq[p];
      const int ti = tgt[q];
      const float aq = al[q], de = s_de[q];
      const float4* xr4 = reinterpret_cast<const float4*>(s_rows + ti * HV);
      const float4* g4 = reinterpret_cast<const float4*>(s_g + ti * HV);
#pragma unroll
      for (int v = 0; v < HV / 4; ++v) {
        const float4 fr = xr4[v], fg = g4[v];
        const float zr[4] = {fr.x, fr.y, fr.z, fr.w}, gg[4] = {fg.x, fg.y, fg.z, fg.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * v + e;
          const float z = xlj[c] + zr[e];
          s[c] += aq * gg[e] + de * a_[c] * (z > 0.f ? 1.f : kLwSlope);
        }
      }
    }
  }
  __syncthreads();  // every lane is done gathering x_r / g rows
  if (i < P) {      // rows >= n carry zeros
    lw_put_row<HV>(s_rows, i, s);
    lw_put_row<HV>(s_g, i, d1);
  }
  __syncthreads();
  lw_lds_to_block<HV>(dxl + base, s_rows, NE, H);
  lw_lds_to_block<HV>(dxr + base, s_g, NE, H);
  __syncthreads();
  if (i < P) lw_put_row<HV>(s_rows, i, d2);
  __syncthreads();
  if (vpart) {  // column sums of the d att rows in a fixed order (8 row groups, then the groups)
    const int c = i & 31, gq = i >> 5;
    float cs = 0.f;
    if (c < H)
      for (int r = gq; r < P; r += 8) cs += s_rows[r * HV + c];
    s_g[i] = cs;  // the g image is free (copied out above)
    __syncthreads();
    if (i < H) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += s_g[32 * q + i];
      vpart[(long)b * H + i] = v;
    }
  } else {
    lw_lds_to_block<HV>(datt + base, s_rows, NE, H);
  }
  if (wl) {  // input gradient d x_l W_l + d x_r W_r on the matrix cores (bf16 images over the row images)
    __syncthreads();
    __bf16* img_l = reinterpret_cast<__bf16*>(s_rows);
    __bf16* img_r = reinterpret_cast<__bf16*>(s_g);
    if (i < ((P + 31) & ~31)) {
      lw_put_bf16_row<HV>(img_l, i, s, H);
      lw_put_bf16_row<HV>(img_r, i, d1, H);
    }
    __syncthreads();
    lw_mfma_rows<true>(img_l, wl, nullptr, dh_in, img_r, wr, nullptr, nullptr, P, H, (long)b * P);
  }
}

// Deterministic column sums of x [R, C] (row stride ldx, C <= 256): phase 1 -- block k sums rows
// [k*chunk, (k+1)*chunk): lane t < L = (256 / C) C owns column t % C and rows t / C + j (L / C), so a
// wave reads whole rows (coalesced); the lanes of a column are added in a fixed order.  Phase 2 --
// one block per column, a fixed-shape tree over the part rows (+= when accumulate).
__global__ __launch_bounds__(256) void lw_colsum_p1_kernel(const float* __restrict__ x, long R, int C, long ldx, long chunk,
                                                           float* __restrict__ part) {
  __shared__ float red[256];
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < R ? r0 + chunk : R;
  const int t = threadIdx.x;
  const int rows = 256 / C, L = rows * C;
  float s = 0.f;
  if (t < L) {
    const int c = t % C;
    for (long r = r0 + t / C; r < r1; r += rows) s += x[r * ldx + c];
  }
  red[t] = s;
  __syncthreads();
  if (t < C) {
    float v = 0.f;
    for (int j = t; j < L; j += C) v += red[j];
    part[(long)blockIdx.x * C + t] = v;
  }
}
__global__ __launch_bounds__(256) void lw_colsum_p2_kernel(const float* __restrict__ part, int K, int C, float* out,
                                                           int accumulate) {
  __shared__ float red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  for (int k = t; k < K; k += 256) s += part[(long)k * C + c];
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) out[c] = accumulate ? out[c] + red[0] : red[0];
}

// First conv's node linears from a narrow input (Fi small, e.g. 3 features): x_l = x W_l^T + b_l and
// x_r likewise in one pass (thread = (row, channel); the weights are L1-resident).
__global__ __launch_bounds__(256) void lw_node_linear_kernel(const float* __restrict__ x, long R, int Fi, int H,
                                                             const float* __restrict__ wl, const float* __restrict__ bl,
                                                             const float* __restrict__ wr, const float* __restrict__ br,
                                                             float* __restrict__ xl, float* __restrict__ xr) {
  // 8 rows x 32 channel lanes (4 x 64 for H > 32) per block step (no per-element 64-bit division); the
  // lane's weight rows stay in registers (Fi <= 8); consecutive lanes write consecutive channels of a row
  const int lpr = H <= 32 ? 32 : 64, rps = 256 / lpr;
  const int c = threadIdx.x % lpr, rl = threadIdx.x / lpr;
  const bool on = c < H;
  const int cc = on ? c : 0;
  float wlr[8], wrr[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wlr[k] = k < Fi ? wl[cc * Fi + k] : 0.f;
    wrr[k] = k < Fi ? wr[cc * Fi + k] : 0.f;
  }
  const float b0 = bl[cc], b1 = br[cc];
  for (long r = (long)blockIdx.x * rps + rl; r < R; r += (long)gridDim.x * rps) {
    float a = b0, b = b1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < Fi) {
        const float v = x[r * Fi + k];
        a = fmaf(wlr[k], v, a);
        b = fmaf(wrr[k], v, b);
      }
    }
    if (on) {
      xl[r * H + c] = a;
      xr[r * H + c] = b;
    }
  }
}

// All parameter gradients of one conv in one pass over its rows (phase 1; phase 2 = lw_colsum_p2 over
// the C outputs): out = [dW_l = dxl^T h | db_l = 1^T dxl | dW_r = dxr^T h | db_r | d att = 1^T datt |
// d bias = 1^T dy] -- the conv's block layout in the flat gradient.  Block k takes rows
// [k chunk, (k+1) chunk) in stages of LW_RB rows: the five row blocks are contiguous in memory and
// copied to LDS with 16-byte loads; thread t owns outputs t + 256 i and sums the stage rows in order
// (fp32, deterministic).
constexpr int LW_RB = 64;
__device__ __forceinline__ void lw_stage_rows(const float* __restrict__ src, long r0, int nr, int w, float* dst) {
  const float* p = src + r0 * w;
  const int n = nr * w;
  if (((uintptr_t)p & 15) == 0 && ((uintptr_t)dst & 15) == 0 && (n & 3) == 0) {
    for (int k = threadIdx.x; k < (n >> 2); k += 256)
      reinterpret_cast<float4*>(dst)[k] = reinterpret_cast<const float4*>(p)[k];
  } else {
    for (int k = threadIdx.x; k < n; k += 256) dst[k] = p[k];
  }
}

template <int NO>
__global__ __launch_bounds__(256) void lw_conv_grads_kernel(const float* __restrict__ dxl, const float* __restrict__ dxr,
                                                            const float* __restrict__ datt, const float* __restrict__ dy,
                                                            const float* __restrict__ hin, long R, int H, int Fi,
                                                            long chunk, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lw_rows[];  // [dxl | dxr | datt | dy][LW_RB][H], h [LW_RB][Fi]
  const int C = 2 * H * Fi + 4 * H, HF = H * Fi, S = LW_RB * H;
  float* s_h = lw_rows + 4 * S;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < R ? r0 + chunk : R;
  // output o -> (first factor: block + channel, second factor: h column or none)
  int fa[NO], fb[NO];
  float acc[NO];
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    const int o = threadIdx.x + 256 * i;
    acc[i] = 0.f;
    fa[i] = 0;
    fb[i] = -1;
    if (o < HF) { fa[i] = o / Fi; fb[i] = o % Fi; }
    else if (o < HF + H) { fa[i] = o - HF; }
    else if (o < 2 * HF + H) { fa[i] = S + (o - HF - H) / Fi; fb[i] = (o - HF - H) % Fi; }
    else if (o < 2 * HF + 2 * H) { fa[i] = S + (o - 2 * HF - H); }
    else if (o < 2 * HF + 3 * H) { fa[i] = 2 * S + (o - 2 * HF - 2 * H); }
    else if (o < C) { fa[i] = 3 * S + (o - 2 * HF - 3 * H); }
  }
  for (long rb = r0; rb < r1; rb += LW_RB) {
    const int nr = (int)(r1 - rb < LW_RB ? r1 - rb : LW_RB);
    lw_stage_rows(dxl, rb, nr, H, lw_rows);
    lw_stage_rows(dxr, rb, nr, H, lw_rows + S);
    lw_stage_rows(datt, rb, nr, H, lw_rows + 2 * S);
    lw_stage_rows(dy, rb, nr, H, lw_rows + 3 * S);
    lw_stage_rows(hin, rb, nr, Fi, s_h);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      if ((int)threadIdx.x + 256 * i < C) {
        float a = acc[i];
        const float* pa = lw_rows + fa[i];
        if (fb[i] >= 0) {
          const float* pb = s_h + fb[i];
          for (int row = 0; row < nr; ++row) a += pa[row * H] * pb[row * Fi];
        } else {
          for (int row = 0; row < nr; ++row) a += pa[row * H];
        }
        acc[i] = a;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    const int o = threadIdx.x + 256 * i;
    if (o < C) part[(long)blockIdx.x * C + o] = acc[i];
  }
}

// MFMA variant (H, Fi <= 32): the same outputs and partial layout.  Per stage of LW_RB rows, wave w owns rows
// [16w, 16w + 16) and accumulates dW_l = dxl^T h and dW_r = dxr^T h on the matrix cores (A = the 16 rows'
// d x column for channel c = lane, B = their h column for input k = lane; bf16 operands, fp32 accumulation);
// the four vector sums (db_l, db_r, d att, d bias) stay fp32 on the VALU.  The waves' tiles are added in a
// fixed order at the end (deterministic).
__global__ __launch_bounds__(256) void lw_conv_grads_mfma_kernel(const float* __restrict__ dxl, const float* __restrict__ dxr,
                                                                 const float* __restrict__ datt, const float* __restrict__ dy,
                                                                 const float* __restrict__ hin, long R, int H, int Fi,
                                                                 long chunk, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lw_rows[];  // [dxl | dxr | datt | dy][LW_RB][H], h [LW_RB][Fi]
  const int C = 2 * H * Fi + 4 * H, HF = H * Fi, S = LW_RB * H;
  float* s_h = lw_rows + 4 * S;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < R ? r0 + chunk : R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane & 31, hh = lane >> 5;
  f32x16 gl, gr;
  mf_zero(gl);
  mf_zero(gr);
  float vsum = 0.f;  // thread t < 4H: vector output t (db_l, db_r, d att, d bias)
  const int vb = tid / H, vc = tid - vb * H;  // block of [dxl | dxr | datt | dy] and channel
  for (long rb = r0; rb < r1; rb += LW_RB) {
    const int nr = (int)(r1 - rb < LW_RB ? r1 - rb : LW_RB);
    lw_stage_rows(dxl, rb, nr, H, lw_rows);
    lw_stage_rows(dxr, rb, nr, H, lw_rows + S);
    lw_stage_rows(datt, rb, nr, H, lw_rows + 2 * S);
    lw_stage_rows(dy, rb, nr, H, lw_rows + 3 * S);
    lw_stage_rows(hin, rb, nr, Fi, s_h);
    __syncthreads();
    if (tid < 4 * H) {
      const float* pa = lw_rows + vb * S + vc;
      for (int row = 0; row < nr; ++row) vsum += pa[row * H];
    }
    if (16 * wave < nr) {
      bf16x8 al, ar, bh;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = 16 * wave + 8 * hh + j;
        const bool in = row < nr;
        al[j] = (__bf16)((in && c < H) ? lw_rows[row * H + c] : 0.f);
        ar[j] = (__bf16)((in && c < H) ? lw_rows[S + row * H + c] : 0.f);
        bh[j] = (__bf16)((in && c < Fi) ? s_h[row * Fi + c] : 0.f);
      }
      gl = mf_mma(al, bh, gl);
      gr = mf_mma(ar, bh, gr);
    }
    __syncthreads();
  }
  // wave tiles -> LDS [wave][l|r][32][32], summed over the waves in a fixed order
  float* red = lw_rows;  // 4 x 2 x 1024 floats (the stage buffers are free)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = mf_row(i, hh);  // dW row = channel of the A operand (row of the 32x32 tile)
    red[(wave * 2 + 0) * 1024 + row * 32 + c] = gl[i];
    red[(wave * 2 + 1) * 1024 + row * 32 + c] = gr[i];
  }
  __syncthreads();
  for (int o = tid; o < 2 * HF; o += 256) {
    const int side = o >= HF, oo = o - side * HF, ch = oo / Fi, k = oo - ch * Fi;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + side) * 1024 + ch * 32 + k];
    part[(long)blockIdx.x * C + (side ? HF + H + oo : oo)] = v;  // [dW_l | db_l | dW_r | db_r | att | bias]
  }
  if (tid < 4 * H) {
    const int off = vb == 0 ? HF : vb == 1 ? 2 * HF + H : 2 * HF + 2 * H + (vb - 2) * H;
    part[(long)blockIdx.x * C + off + vc] = vsum;
  }
}

// Conv parameter gradients streamed from HBM (H <= 32, Fi <= 31): dW = dX^T h on the matrix cores with the
// A / B fragments loaded straight from the row-major [R][H] / [R][Fi] blocks (lane c = channel, 8 rows per
// lane half) and h extended by a ones column (k = Fi), so the same MFMA also yields the bias sums of d x_l /
// d x_r; the d bias sum of dY on the VALU.  Each wave walks 16-row steps of its workgroup's contiguous row
// range with the next step's loads in flight (no LDS staging round trip per step); the 4 waves' tiles are
// combined in a fixed order into one partial row per workgroup [dW_l | db_l | dW_r | db_r | 0 | d bias]
// (d att comes from the attention backward's per-graph sums).  Deterministic.
__global__ __launch_bounds__(256) void lw_conv_grads_stream_kernel(const float* __restrict__ dxl,
                                                                   const float* __restrict__ dxr,
                                                                   const float* __restrict__ dy,
                                                                   const float* __restrict__ hin, long R, int H, int Fi,
                                                                   long rows_per_blk, float* __restrict__ part) {
  __shared__ float red[4][2][32][33];
  __shared__ float redb[4][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, hh = lane >> 5;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = r0 + rows_per_blk < R ? r0 + rows_per_blk : R;
  f32x16 gl, gr;
  mf_zero(gl);
  mf_zero(gr);
  float vb = 0.f;
  const bool ch = c < H, hk = c < Fi, one = c == Fi;
  // every load issued unconditionally at a clamped address into raw registers; the range masks are applied
  // where the values are consumed (a branch around a load, or a select right after it, made the compiler
  // wait for the outstanding loads there: one step in flight)
  const int cc = ch ? c : H - 1, ck = hk ? c : Fi - 1;
  auto load = [&](long rs, float (&l)[8], float (&q)[8], float (&h)[8], float (&y)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      long v = rs + 8 * hh + j;
      v = v < r1 ? v : r1 - 1;
      l[j] = dxl[v * H + cc];
      q[j] = dxr[v * H + cc];
      y[j] = dy[v * H + cc];
      h[j] = hin[v * Fi + ck];
    }
  };
  auto step = [&](long rs, const float (&l)[8], const float (&q)[8], const float (&h)[8], const float (&y)[8]) {
    bf16x8 al, ar, bh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in = rs + 8 * hh + j < r1;
      al[j] = (__bf16)((in && ch) ? l[j] : 0.f);
      ar[j] = (__bf16)((in && ch) ? q[j] : 0.f);
      bh[j] = (__bf16)(in ? (hk ? h[j] : (one ? 1.f : 0.f)) : 0.f);
      vb += (in && ch) ? y[j] : 0.f;
    }
    gl = mf_mma(al, bh, gl);
    gr = mf_mma(ar, bh, gr);
  };
  // two register sets in a ping-pong: one step computes while the next step's loads are in flight (loads past
  // the range read the last row again and are masked off)
  float l0[8], q0[8], h0[8], y0[8], l1[8], q1[8], h1[8], y1[8];
  long rs = r0 + 16 * w;
  load(rs, l0, q0, h0, y0);
  for (; rs < r1; rs += 128) {
    load(rs + 64, l1, q1, h1, y1);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the conversions the scheduler would hoist
    step(rs, l0, q0, h0, y0);
    load(rs + 128, l0, q0, h0, y0);
    __builtin_amdgcn_sched_barrier(0);
    step(rs + 64, l1, q1, h1, y1);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = mf_row(i, hh);  // output channel (A row); column c = h column k
    red[w][0][row][c] = gl[i];
    red[w][1][row][c] = gr[i];
  }
  vb += __shfl_xor(vb, 32);
  if (hh == 0) redb[w][c] = vb;
  __syncthreads();
  const int HF = H * Fi, C = 2 * HF + 4 * H;
  for (int o = tid; o < C; o += 256) {
    float v = 0.f;
    if (o < 2 * HF + 2 * H) {
      const int side = o >= HF + H, oo = o - side * (HF + H);
      const int chn = oo < HF ? oo / Fi : oo - HF, k = oo < HF ? oo - (oo / Fi) * Fi : Fi;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) v += red[ww][side][chn][k];
    } else if (o >= 2 * HF + 3 * H) {
      const int chn = o - 2 * HF - 3 * H;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) v += redb[ww][chn];
    }
    part[(long)blockIdx.x * C + o] = v;
  }
}

void lw_colsum(uintptr_t x, long R, int C, long ldx, uintptr_t part, uintptr_t out, int accumulate, uintptr_t stream);

// part >= 1024 (2 H Fi + 4 H) floats, vpart [B][H] per-graph d att sums (lw_attn_bwd_gather), vscr >= 1024 H
void lw_conv_grads_v(uintptr_t dxl, uintptr_t dxr, uintptr_t dy, uintptr_t hin, long R, int H, int Fi, uintptr_t part,
                     long part_floats, uintptr_t out, int accumulate, uintptr_t vpart, int B, uintptr_t vscr,
                     uintptr_t stream) {
  GSC_CHECK(H <= 32 && Fi <= 31, "lw_conv_grads_v: H <= 32, Fi <= 31");
  const int C = 2 * H * Fi + 4 * H;
  long rpb = (R + 1023) / 1024;
  rpb = (rpb + 63) / 64 * 64;
  const int K = (int)((R + rpb - 1) / rpb);
  GSC_CHECK((long)K * C <= part_floats, "lw_conv_grads_v: partials buffer too small");
  const hipStream_t s = stream_of(stream);
  hipLaunchKernelGGL(lw_conv_grads_stream_kernel, dim3(K), dim3(256), 0, s, ptr<const float>(dxl),
                     ptr<const float>(dxr), ptr<const float>(dy), ptr<const float>(hin), R, H, Fi, rpb, ptr<float>(part));
  check_launch();
  hipLaunchKernelGGL(lw_colsum_p2_kernel, dim3(C), dim3(256), 0, s, ptr<const float>(part), K, C, ptr<float>(out),
                     accumulate);
  check_launch();
  // d att: the per-graph sums on top (the partial rows carry zeros there)
  lw_colsum(vpart, B, H, H, vscr, out + sizeof(float) * (2 * H * Fi + 2 * H), 1, stream);
}

// ---------------------------------------------------------------------------------------------------
static LwGraph lw_graph(py::dict t, uintptr_t topo, int B, int P, int H) {
  LwGraph g{};
  g.topo = ptr<const int32_t>(topo);
  g.nnodes = ptr<const int32_t>(t["nnodes"].cast<uintptr_t>());
  g.in_ptr = ptr<const int32_t>(t["in_ptr"].cast<uintptr_t>());
  g.in_src = ptr<const int32_t>(t["in_src"].cast<uintptr_t>());
  g.out_ptr = ptr<const int32_t>(t["out_ptr"].cast<uintptr_t>());
  g.out_q = ptr<const int32_t>(t["out_q"].cast<uintptr_t>());
  g.deg = ptr<const float>(t["deg"].cast<uintptr_t>());
  g.M = t["M"].cast<int>();
  g.B = B;
  g.P = P;
  g.H = H;
  GSC_CHECK(H <= 64, "layer-wise GATv2: at most 64 channels");
  return g;
}

// lanes per node: a half-wave for H <= 32 (two nodes per wave), a whole wave up to 64 channels
static int lanes_per_node(const LwGraph& g) { return g.H <= 32 ? 32 : 64; }
static dim3 node_grid(const LwGraph& g) {
  const long per = 256 / lanes_per_node(g);
  return dim3((unsigned)(((long)g.B * g.P + per - 1) / per));
}

// next = (wl, bl, wr, br, xl_out, xr_out) of the following conv (H -> H), or () for the last conv
void lw_pool(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t h, uintptr_t emb, uintptr_t stream);

// emb (last conv, optional): also the mean pool into emb [B][H] (fused on the lane-per-node path)
// store: bit 0 = the output rows h_out, bit 1 = alpha are needed (a later backward); the staged kernel skips
// the others, the other kernels always write both
// first = (x, Fi, wl, bl, wr, br, store_xlxr): the first conv from its narrow input x [B*P][Fi] (Fi <= 8); x_l /
// x_r go to xl / xr only when store_xlxr (a backward follows) -- or always, through lw_node_linear, when the
// staged kernel does not apply
void lw_node_linear(uintptr_t x, long R, int Fi, int H, uintptr_t wl, uintptr_t bl, uintptr_t wr, uintptr_t br,
                    uintptr_t xl, uintptr_t xr, uintptr_t stream);
void lw_attn_fwd(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t xl, uintptr_t xr, uintptr_t att,
                 uintptr_t bias, int relu, uintptr_t h_out, uintptr_t alpha, uintptr_t stream, py::tuple next,
                 uintptr_t emb, int store, py::tuple first) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  LwFirst f0{};
  if (first.size() == 7) {
    f0.x = ptr<const float>(first[0].cast<uintptr_t>());
    f0.Fi = first[1].cast<int>();
    f0.wl = ptr<const float>(first[2].cast<uintptr_t>());
    f0.bl = ptr<const float>(first[3].cast<uintptr_t>());
    f0.wr = ptr<const float>(first[4].cast<uintptr_t>());
    f0.br = ptr<const float>(first[5].cast<uintptr_t>());
    if (first[6].cast<int>()) {
      f0.xl_out = ptr<float>(xl);
      f0.xr_out = ptr<float>(xr);
    }
    GSC_CHECK(f0.Fi >= 1 && f0.Fi <= 8, "lw_attn_fwd: the fused first conv takes Fi <= 8 input features");
  } else {
    GSC_CHECK(first.size() == 0, "lw_attn_fwd: first = (x, Fi, wl, bl, wr, br, store_xlxr) or ()");
  }
  // the non-staged kernels read x_l / x_r from memory
  auto materialise_first = [&]() {
    if (f0.x)
      lw_node_linear(reinterpret_cast<uintptr_t>(f0.x), (long)B * P, f0.Fi, H, reinterpret_cast<uintptr_t>(f0.wl),
                     reinterpret_cast<uintptr_t>(f0.bl), reinterpret_cast<uintptr_t>(f0.wr),
                     reinterpret_cast<uintptr_t>(f0.br), xl, xr, stream);
  };
  LwNext nx{};
  if (next.size() == 6) {
    nx.wl = ptr<const float>(next[0].cast<uintptr_t>());
    nx.bl = ptr<const float>(next[1].cast<uintptr_t>());
    nx.wr = ptr<const float>(next[2].cast<uintptr_t>());
    nx.br = ptr<const float>(next[3].cast<uintptr_t>());
    nx.xl = ptr<float>(next[4].cast<uintptr_t>());
    nx.xr = ptr<float>(next[5].cast<uintptr_t>());
  } else {
    GSC_CHECK(next.size() == 0, "lw_attn_fwd: next = (wl, bl, wr, br, xl, xr) or ()");
  }
  if (H <= 32) {  // lane per node
    const int hv = H <= 8 ? 8 : H <= 16 ? 16 : H <= 24 ? 24 : 32;
    // GSC_LW_MFMA=0: the lane kernels (VALU node linears) even where the staged kernel applies
    static const bool mf_env = getenv("GSC_LW_MFMA") == nullptr || atoi(getenv("GSC_LW_MFMA")) != 0;
    // staged variant: both row blocks in LDS, coalesced output / alpha stores, MFMA linears
    const size_t lds_st = sizeof(float) * ((size_t)P * (hv + 4) + 2 * g.M + 2 * P + 1);
    if (mf_env && P <= 256 && hv >= 16 && (!nx.wl || lw_mfma_fits(P, hv + 4)) && lds_st <= 80 * 1024) {
      auto ks = f0.x ? (hv == 16 ? lw_stage_attn_fwd_kernel<16, true>
                                 : hv == 24 ? lw_stage_attn_fwd_kernel<24, true> : lw_stage_attn_fwd_kernel<32, true>)
                     : (hv == 16 ? lw_stage_attn_fwd_kernel<16> : hv == 24 ? lw_stage_attn_fwd_kernel<24>
                                                                        : lw_stage_attn_fwd_kernel<32>);
      if (lds_st > 65536)  // two workgroups still share a CU's 160 KB
        GSC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(ks),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_st));
      hipLaunchKernelGGL(ks, dim3(B), dim3(256), lds_st, stream_of(stream), g, ptr<const float>(xl),
                         ptr<const float>(xr), ptr<const float>(att), ptr<const float>(bias), relu,
                         (store & 1) ? ptr<float>(h_out) : nullptr, (store & 2) ? ptr<float>(alpha) : nullptr, nx,
                         ptr<float>(emb), f0);
      check_launch();
      return;
    }
    materialise_first();
    // lane kernel: H < 16 channels, graphs whose rows do not tile the staged kernel's MFMA image (P % 32 != 0
    // at H = 16), GSC_LW_MFMA=0, n_pad > 256
    const size_t lds = sizeof(float) * ((size_t)P * hv + (nx.wl ? 2 * H * hv : 0) + 2 * g.M + 2 * P + 1);
    if (lds <= 64 * 1024) {
      auto kl = hv == 8 ? lw_lane_attn_fwd_kernel<8>
                : hv == 16 ? lw_lane_attn_fwd_kernel<16> : hv == 24 ? lw_lane_attn_fwd_kernel<24>
                                                           : lw_lane_attn_fwd_kernel<32>;
      hipLaunchKernelGGL(kl, dim3(B), dim3(256), lds, stream_of(stream), g, ptr<const float>(xl), ptr<const float>(xr),
                         ptr<const float>(att), ptr<const float>(bias), relu, ptr<float>(h_out), ptr<float>(alpha), nx,
                         ptr<float>(emb));
      check_launch();
      return;
    }
  }
  if (H > 32) materialise_first();
  const size_t graph_lds = sizeof(float) * (2L * P * H + (nx.wl ? 2L * H * H : 0) + (P + 1) + g.M + P);
  if (graph_lds <= 64 * 1024) {  // per-graph blocks (>= 2 workgroups per CU)
    auto kg = lanes_per_node(g) == 32 ? lw_graph_attn_fwd_kernel<32> : lw_graph_attn_fwd_kernel<64>;
    hipLaunchKernelGGL(kg, dim3(B), dim3(256), graph_lds, stream_of(stream), g, ptr<const float>(xl),
                       ptr<const float>(xr), ptr<const float>(att), ptr<const float>(bias), relu, ptr<float>(h_out),
                       ptr<float>(alpha), nx);
    check_launch();
    if (emb) lw_pool(tables, topo, B, P, H, h_out, emb, stream);
    return;
  }
  const size_t lds = nx.wl ? 2 * sizeof(float) * H * H : 0;
  auto k = lanes_per_node(g) == 32 ? lw_attn_fwd_kernel<32> : lw_attn_fwd_kernel<64>;
  hipLaunchKernelGGL(k, node_grid(g), dim3(256), lds, stream_of(stream), g, ptr<const float>(xl),
                     ptr<const float>(xr), ptr<const float>(att), ptr<const float>(bias), relu, ptr<float>(h_out),
                     ptr<float>(alpha), nx);
  check_launch();
  if (emb) lw_pool(tables, topo, B, P, H, h_out, emb, stream);
}

void lw_pool(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t h, uintptr_t emb, uintptr_t stream) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  const int per = 256 / lanes_per_node(g);
  auto k = per == 8 ? lw_pool_kernel<32> : lw_pool_kernel<64>;
  hipLaunchKernelGGL(k, dim3((B + per - 1) / per), dim3(256), 0, stream_of(stream), g, ptr<const float>(h),
                     ptr<float>(emb));
  check_launch();
}

void lw_pool_bwd(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t demb, uintptr_t dh, uintptr_t stream) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  const long total = (long)B * P * H;
  hipLaunchKernelGGL(lw_pool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream_of(stream), g,
                     ptr<const float>(demb), ptr<float>(dh));
  check_launch();
}

void lw_attn_bwd(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t dh, uintptr_t h_out, uintptr_t xl,
                 uintptr_t xr, uintptr_t alpha, uintptr_t att, uintptr_t dxr, uintptr_t msg, uintptr_t datt,
                 uintptr_t stream) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  auto k = lanes_per_node(g) == 32 ? lw_attn_bwd_kernel<32> : lw_attn_bwd_kernel<64>;
  hipLaunchKernelGGL(k, node_grid(g), dim3(256), 0, stream_of(stream), g, ptr<float>(dh),
                     ptr<const float>(h_out), ptr<const float>(xl), ptr<const float>(xr), ptr<const float>(alpha),
                     ptr<const float>(att), ptr<float>(dxr), ptr<float>(msg), ptr<float>(datt));
  check_launch();
}

// wl/wr (H x H, 0 = skip): also dh = dxl W_l + dxr W_r (input gradient of a conv with H inputs)
void lw_src_gather(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t msg, uintptr_t dxl, uintptr_t stream,
                   uintptr_t dxr, uintptr_t wl, uintptr_t wr, uintptr_t dh) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  GSC_CHECK(!wl || (dxr && wr && dh), "lw_src_gather: the input gradient needs dxr, wl, wr, dh");
  auto k = lanes_per_node(g) == 32 ? lw_src_gather_kernel<32> : lw_src_gather_kernel<64>;
  const size_t lds = wl ? 2 * sizeof(float) * H * H : 0;
  hipLaunchKernelGGL(k, node_grid(g), dim3(256), lds, stream_of(stream), g, ptr<const float>(msg), ptr<float>(dxl),
                     ptr<const float>(dxr), ptr<const float>(wl), ptr<const float>(wr), ptr<float>(dh));
  check_launch();
}

// attention backward + source gather (+ input gradient when wl): one per-graph launch when the
// graph's x_l block fits the LDS budget, else the per-node kernels
// vpart (optional, [B][H]): the staged kernel writes per-graph d att sums there instead of the d att rows;
// returns whether it did (else the rows are in datt)
// demb (optional, [B][H]): dh is the mean-pool backward of demb (the last conv): formed inside the staged
// kernel, or written to dh by lw_pool_bwd first when another kernel runs
void lw_pool_bwd(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t demb, uintptr_t dh, uintptr_t stream);
bool lw_attn_bwd_gather(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t dh, uintptr_t h_out, uintptr_t xl,
                        uintptr_t xr, uintptr_t alpha, uintptr_t att, uintptr_t dxr, uintptr_t msg, uintptr_t datt,
                        uintptr_t dxl, uintptr_t wl, uintptr_t wr, uintptr_t dh_in, uintptr_t stream, uintptr_t vpart,
                        uintptr_t demb) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
  GSC_CHECK(!wl || (wr && dh_in), "lw_attn_bwd_gather: the input gradient needs wl, wr, dh_in");
  if (H <= 32) {  // lane per node
    const int hv = H <= 8 ? 8 : H <= 16 ? 16 : H <= 24 ? 24 : 32;
    static const bool mf_env = getenv("GSC_LW_MFMA") == nullptr || atoi(getenv("GSC_LW_MFMA")) != 0;
    const bool mf = mf_env && wl && lw_mfma_fits(P, hv);
    // staged: two row images + fp32 alpha / de + u16 / u8 message indices; 16-B aligned [P][H] blocks
    const size_t lst = sizeof(float) * (2 * (size_t)P * hv + 2 * g.M + P + 2 * (P + 1)) + 4 * (size_t)g.M;
    auto al16 = [](uintptr_t p) { return (p & 15) == 0; };
    const bool blocks16 = ((long)P * H) % 4 == 0 && al16(dh) && al16(xl) && al16(xr) && (!h_out || al16(h_out)) &&
                          al16(dxr) && al16(datt) && al16(dxl);
    if (mf_env && P <= 256 && hv >= 16 && g.M < 65536 && blocks16 && (!wl || lw_mfma_fits(P, hv)) &&
        lst <= 80 * 1024) {
      auto ks = hv == 16 ? lw_stage_attn_bwd_kernel<16> : hv == 24 ? lw_stage_attn_bwd_kernel<24>
                                                                  : lw_stage_attn_bwd_kernel<32>;
      if (lst > 65536)
        GSC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(ks),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lst));
      hipLaunchKernelGGL(ks, dim3(B), dim3(256), lst, stream_of(stream), g, ptr<float>(dh), ptr<const float>(h_out),
                         ptr<const float>(xl), ptr<const float>(xr), ptr<const float>(alpha), ptr<const float>(att),
                         ptr<float>(dxr), ptr<float>(datt), ptr<float>(dxl), ptr<const float>(wl),
                         ptr<const float>(wr), ptr<float>(dh_in), ptr<float>(vpart), ptr<const float>(demb));
      check_launch();
      return vpart != 0;
    }
    if (demb) lw_pool_bwd(tables, topo, B, P, H, demb, dh, stream);
    demb = 0;
    const size_t ll = sizeof(float) * (2 * (size_t)P * hv + (wl && !mf ? 2 * H * hv : 0) + 5 * g.M + P + 2 * (P + 1));
    if (ll <= 80 * 1024) {  // >= 2 workgroups per CU
      auto kl = mf ? (hv == 16 ? lw_lane_attn_bwd_kernel<16, true> : hv == 24 ? lw_lane_attn_bwd_kernel<24, true>
                                                                    : lw_lane_attn_bwd_kernel<32, true>)
                   : hv == 8 ? lw_lane_attn_bwd_kernel<8>
                   : hv == 16 ? lw_lane_attn_bwd_kernel<16> : hv == 24 ? lw_lane_attn_bwd_kernel<24>
                                                              : lw_lane_attn_bwd_kernel<32>;
      hipLaunchKernelGGL(kl, dim3(B), dim3(256), ll, stream_of(stream), g, ptr<float>(dh), ptr<const float>(h_out),
                         ptr<const float>(xl), ptr<const float>(xr), ptr<const float>(alpha), ptr<const float>(att),
                         ptr<float>(dxr), ptr<float>(datt), ptr<float>(dxl), ptr<const float>(wl),
                         ptr<const float>(wr), ptr<float>(dh_in));
      check_launch();
      return false;
    }
  }
  if (demb) lw_pool_bwd(tables, topo, B, P, H, demb, dh, stream);
  const size_t lds = sizeof(float) * ((size_t)P * H + (wl ? 2 * H * H : 0) + g.M + P + 2 * (P + 1) + 2 * g.M);
  if (lds <= 64 * 1024) {
    auto k = lanes_per_node(g) == 32 ? lw_graph_attn_bwd_kernel<32> : lw_graph_attn_bwd_kernel<64>;
    hipLaunchKernelGGL(k, dim3(B), dim3(256), lds, stream_of(stream), g, ptr<float>(dh), ptr<const float>(h_out),
                       ptr<const float>(xl), ptr<const float>(xr), ptr<const float>(alpha), ptr<const float>(att),
                       ptr<float>(dxr), ptr<float>(msg), ptr<float>(datt), ptr<float>(dxl), ptr<const float>(wl),
                       ptr<const float>(wr), ptr<float>(dh_in));
    check_launch();
    return false;
  }
  lw_attn_bwd(tables, topo, B, P, H, dh, h_out, xl, xr, alpha, att, dxr, msg, datt, stream);
  lw_src_gather(tables, topo, B, P, H, msg, dxl, stream, dxr, wl, wr, dh_in);
  return false;
}

void lw_relu_mask(uintptr_t dh, uintptr_t h, long n, uintptr_t stream) {
  hipLaunchKernelGGL(lw_relu_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream_of(stream),
                     ptr<float>(dh), ptr<const float>(h), n);
  check_launch();
}

// part must hold >= min(R, 1024) x C floats
void lw_colsum(uintptr_t x, long R, int C, long ldx, uintptr_t part, uintptr_t out, int accumulate, uintptr_t stream) {
  GSC_CHECK(C >= 1 && C <= 256, "lw_colsum: 1..256 columns");
  const long chunk = R <= 1024 ? 1 : (R + 1023) / 1024;
  const int K = (int)((R + chunk - 1) / chunk);
  hipLaunchKernelGGL(lw_colsum_p1_kernel, dim3(K), dim3(256), 0, stream_of(stream), ptr<const float>(x), R, C, ldx, chunk,
                     ptr<float>(part));
  hipLaunchKernelGGL(lw_colsum_p2_kernel, dim3(C), dim3(256), 0, stream_of(stream), ptr<const float>(part), K, C,
                     ptr<float>(out), accumulate);
  check_launch();
}

void lw_node_linear(uintptr_t x, long R, int Fi, int H, uintptr_t wl, uintptr_t bl, uintptr_t wr, uintptr_t br,
                    uintptr_t xl, uintptr_t xr, uintptr_t stream) {
  GSC_CHECK(Fi <= 8 && H <= 64, "lw_node_linear: Fi <= 8, H <= 64");
  long g = (R + 3) / 4;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(lw_node_linear_kernel, dim3((unsigned)g), dim3(256), 0, stream_of(stream), ptr<const float>(x), R, Fi,
                     H, ptr<const float>(wl), ptr<const float>(bl), ptr<const float>(wr), ptr<const float>(br),
                     ptr<float>(xl), ptr<float>(xr));
  check_launch();
}

// part must hold >= min(R, 1024) x (2 H Fi + 4 H) floats; out = the conv's gradient block
void lw_conv_grads(uintptr_t dxl, uintptr_t dxr, uintptr_t datt, uintptr_t dy, uintptr_t hin, long R, int H, int Fi,
                   uintptr_t part, long part_floats, uintptr_t out, int accumulate, uintptr_t stream) {
  const int C = 2 * H * Fi + 4 * H;
  const long chunk = R <= 1024 ? 1 : (R + 1023) / 1024;
  const int K = (int)((R + chunk - 1) / chunk);
  GSC_CHECK((long)K * C <= part_floats, "lw_conv_grads: partials buffer too small");
  const int no = (C + 255) / 256;
  const size_t lds = sizeof(float) * LW_RB * (4 * H + Fi);  // 4 S is a multiple of 4 floats: s_h stays aligned
  const hipStream_t s = stream_of(stream);
  static const bool mf_env = getenv("GSC_LW_MFMA") == nullptr || atoi(getenv("GSC_LW_MFMA")) != 0;
  if (mf_env && H <= 32 && Fi <= 32 && 4 * H <= 256) {  // dW on the matrix cores
    const size_t lds_mf = std::max(lds, sizeof(float) * 8 * 1024);  // the final wave-tile reduction
    hipLaunchKernelGGL(lw_conv_grads_mfma_kernel, dim3(K), dim3(256), lds_mf, s, ptr<const float>(dxl),
                       ptr<const float>(dxr), ptr<const float>(datt), ptr<const float>(dy), ptr<const float>(hin), R, H,
                       Fi, chunk, ptr<float>(part));
    check_launch();
    hipLaunchKernelGGL(lw_colsum_p2_kernel, dim3(C), dim3(256), 0, s, ptr<const float>(part), K, C, ptr<float>(out),
                       accumulate);
    check_launch();
    return;
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(K), dim3(256), lds, s, ptr<const float>(dxl), ptr<const float>(dxr),
                       ptr<const float>(datt), ptr<const float>(dy), ptr<const float>(hin), R, H, Fi, chunk,
                       ptr<float>(part));
  };
  if (no <= 1) go(lw_conv_grads_kernel<1>);
  else if (no <= 2) go(lw_conv_grads_kernel<2>);
  else if (no <= 5) go(lw_conv_grads_kernel<5>);
  else if (no <= 9) go(lw_conv_grads_kernel<9>);
  else if (no <= 17) go(lw_conv_grads_kernel<17>);
  else {
    GSC_CHECK(no <= 36, "lw_conv_grads: at most 64 channels");
    go(lw_conv_grads_kernel<36>);
  }
  check_launch();
  hipLaunchKernelGGL(lw_colsum_p2_kernel, dim3(C), dim3(256), 0, s, ptr<const float>(part), K, C, ptr<float>(out),
                     accumulate);
  check_launch();
}

void register_gnn_lw(py::module_& m) {
  m.def("lw_node_linear", &lw_node_linear, "layer-wise GATv2: first conv's node linears (narrow input)");
  m.def("lw_conv_grads", &lw_conv_grads, "layer-wise GATv2: every parameter gradient of one conv (one pass)");
  m.def("lw_attn_fwd", &lw_attn_fwd, "layer-wise GATv2: attention + aggregation (+ReLU), alpha saved; optionally "
        "the next conv's node linears", py::arg("tables"), py::arg("topo"), py::arg("B"), py::arg("P"), py::arg("H"),
        py::arg("xl"), py::arg("xr"), py::arg("att"), py::arg("bias"), py::arg("relu"), py::arg("h_out"),
        py::arg("alpha"), py::arg("stream"), py::arg("next") = py::tuple(), py::arg("emb") = 0, py::arg("store") = 3,
        py::arg("first") = py::tuple());
  m.def("lw_pool", &lw_pool, "layer-wise GATv2: mean pool over real nodes");
  m.def("lw_pool_bwd", &lw_pool_bwd, "layer-wise GATv2: mean-pool backward");
  m.def("lw_attn_bwd", &lw_attn_bwd, "layer-wise GATv2: attention backward per target node");
  m.def("lw_src_gather", &lw_src_gather, "layer-wise GATv2: d x_l gathered per source node (+ the input gradient)",
        py::arg("tables"), py::arg("topo"), py::arg("B"), py::arg("P"), py::arg("H"), py::arg("msg"), py::arg("dxl"),
        py::arg("stream"), py::arg("dxr") = 0, py::arg("wl") = 0, py::arg("wr") = 0, py::arg("dh") = 0);
  m.def("lw_relu_mask", &lw_relu_mask, "dh *= (h > 0)");
  m.def("lw_attn_bwd_gather", &lw_attn_bwd_gather,
        "layer-wise GATv2: attention backward + source gather (+ input gradient), per graph when it fits; "
        "returns whether vpart holds the per-graph d att sums", py::arg("tables"), py::arg("topo"), py::arg("B"),
        py::arg("P"), py::arg("H"), py::arg("dh"), py::arg("h_out"), py::arg("xl"), py::arg("xr"), py::arg("alpha"),
        py::arg("att"), py::arg("dxr"), py::arg("msg"), py::arg("datt"), py::arg("dxl"), py::arg("wl"), py::arg("wr"),
        py::arg("dh_in"), py::arg("stream"), py::arg("vpart") = 0, py::arg("demb") = 0);
  m.def("lw_conv_grads_v", &lw_conv_grads_v, "layer-wise GATv2: conv parameter gradients, streamed (MFMA dW with "
        "a ones column for the bias sums), d att from per-graph sums");
  m.def("lw_colsum", &lw_colsum, "deterministic column sums (two phases)");
}

}  // namespace gsc
