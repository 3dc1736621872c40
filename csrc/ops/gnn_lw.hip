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

namespace py = pybind11;

namespace gsc {

constexpr float kLwSlope = 0.2f;

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
  float mx = -__builtin_inff(), den = 0.f, acc = 0.f;
  for (int q = q0; q < q1; ++q) {
    const float xlj = c < H ? xlb[(long)src[q] * H + c] : 0.f;
    const float s = lw_sum<NL>(ac * leaky(xlj + xri));
    if (c == ((q - q0) & (NL - 1))) al[q] = s;  // every lane holds s (xor butterfly)
    if (s > mx) {
      const float r = __expf(mx - s);  // 0 on the first message (mx = -inf)
      den *= r;
      acc *= r;
      mx = s;
    }
    const float e = __expf(s - mx);
    den += e;
    acc += e * xlj;
  }
  const float inv = 1.f / (den + 1e-16f);
  // each lane rescales the scores it stored itself
  for (int q = q0 + c; q < q1; q += NL) al[q] = __expf(al[q] - mx) * inv;
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
  // sum_q' alpha_q' dalpha_q'
  float sad = 0.f;
  for (int q = q0; q < q1; ++q) {
    const int j = src[q];
    const float da = lw_sum<NL>(ch ? gc * xlb[(long)j * H + c] : 0.f);
    sad += al[q] * da;
  }
  float dxr_acc = 0.f, datt_acc = 0.f;
  for (int q = q0; q < q1; ++q) {
    const int j = src[q];
    const float xlj = ch ? xlb[(long)j * H + c] : 0.f;
    const float da = lw_sum<NL>(gc * xlj);
    const float de = al[q] * (da - sad);
    const float z = xlj + xri;
    datt_acc += de * leaky(z);
    const float dz = de * ac * (z > 0.f ? 1.f : kLwSlope);
    dxr_acc += dz;
    if (ch) mb[(long)q * H + c] = al[q] * gc + dz;
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
  const long node = (long)blockIdx.x * (256 / NL) + (threadIdx.x / NL);
  const int c = threadIdx.x & (NL - 1);
  if (node >= (long)g.B * g.P) return;  // whole node groups exit together
  const int H = g.H;
  const int b = (int)(node / g.P), j = (int)(node - (long)b * g.P);
  const int t = g.topo[b];
  float s = 0.f;
  if (j < g.nnodes[t] && c < H) {
    const int p0 = g.out_ptr[(long)t * (g.P + 1) + j], p1 = g.out_ptr[(long)t * (g.P + 1) + j + 1];
    const int32_t* oq = g.out_q + (long)t * g.M;
    const float* mb = msg + (long)b * g.M * H;
    for (int p = p0; p < p1; ++p) s += mb[(long)oq[p] * H + c];
  }
  if (c < H) dxl[node * H + c] = s;
  if (wl) {
    const float r = c < H ? dxr[node * H + c] : 0.f;
    const int cc = c < H ? c : 0;
    float d = 0.f;
    for (int k = 0; k < H; ++k) {
      const float lk = __shfl(s, k, NL), rk = __shfl(r, k, NL);
      d += lk * wl[k * H + cc] + rk * wr[k * H + cc];
    }
    if (c < H) dh[node * H + c] = d;
  }
}

// dh[r, :] *= (h[r, :] > 0)  (ReLU of the layer below; h = that layer's output)
__global__ __launch_bounds__(256) void lw_relu_mask_kernel(float* dh, const float* h, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !(h[i] > 0.f)) dh[i] = 0.f;
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
void lw_attn_fwd(py::dict tables, uintptr_t topo, int B, int P, int H, uintptr_t xl, uintptr_t xr, uintptr_t att,
                 uintptr_t bias, int relu, uintptr_t h_out, uintptr_t alpha, uintptr_t stream, py::tuple next) {
  const LwGraph g = lw_graph(tables, topo, B, P, H);
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
  const size_t lds = nx.wl ? 2 * sizeof(float) * H * H : 0;
  auto k = lanes_per_node(g) == 32 ? lw_attn_fwd_kernel<32> : lw_attn_fwd_kernel<64>;
  hipLaunchKernelGGL(k, node_grid(g), dim3(256), lds, stream_of(stream), g, ptr<const float>(xl),
                     ptr<const float>(xr), ptr<const float>(att), ptr<const float>(bias), relu, ptr<float>(h_out),
                     ptr<float>(alpha), nx);
  check_launch();
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
  hipLaunchKernelGGL(k, node_grid(g), dim3(256), 0, stream_of(stream), g, ptr<const float>(msg), ptr<float>(dxl),
                     ptr<const float>(dxr), ptr<const float>(wl), ptr<const float>(wr), ptr<float>(dh));
  check_launch();
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

void register_gnn_lw(py::module_& m) {
  m.def("lw_attn_fwd", &lw_attn_fwd, "layer-wise GATv2: attention + aggregation (+ReLU), alpha saved; optionally "
        "the next conv's node linears", py::arg("tables"), py::arg("topo"), py::arg("B"), py::arg("P"), py::arg("H"),
        py::arg("xl"), py::arg("xr"), py::arg("att"), py::arg("bias"), py::arg("relu"), py::arg("h_out"),
        py::arg("alpha"), py::arg("stream"), py::arg("next") = py::tuple());
  m.def("lw_pool", &lw_pool, "layer-wise GATv2: mean pool over real nodes");
  m.def("lw_pool_bwd", &lw_pool_bwd, "layer-wise GATv2: mean-pool backward");
  m.def("lw_attn_bwd", &lw_attn_bwd, "layer-wise GATv2: attention backward per target node");
  m.def("lw_src_gather", &lw_src_gather, "layer-wise GATv2: d x_l gathered per source node (+ the input gradient)",
        py::arg("tables"), py::arg("topo"), py::arg("B"), py::arg("P"), py::arg("H"), py::arg("msg"), py::arg("dxl"),
        py::arg("stream"), py::arg("dxr") = 0, py::arg("wl") = 0, py::arg("wr") = 0, py::arg("dh") = 0);
  m.def("lw_relu_mask", &lw_relu_mask, "dh *= (h > 0)");
  m.def("lw_colsum", &lw_colsum, "deterministic column sums (two phases)");
}

}  // namespace gsc
