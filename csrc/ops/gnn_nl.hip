// Node-lane GATv2 embedder forward (gfx950, wave64): one lane per graph node.
//
// A wave holds G = 64 / NP graphs (NP = node slots per graph, e.g. 11 for Abilene -> 5 graphs);
// lane = slot * NP + v.  Every lane keeps its node's feature vector in VGPRs through all
// convolutions, so there is no LDS working set:
//   * node linears: x_l[c] = b_l[c] + sum_k W_l[c][k] h[k] — W from a zero-padded copy in global
//     memory read with uniform addresses (scalar loads -> SGPR operands of v_fma);
//   * messages (lane = target node i, loop over its in-neighbours j): x_l[j] arrives from lane j
//     via ds_bpermute; score e = att . lrelu(x_l[j] + x_r[i]); softmax and the attention-weighted
//     sum run as one online pass (running max / rescaled sum), then / in-degree + bias (PyG
//     GATv2Conv, aggr='mean', self loops in the topology tables);
//   * mean pool: rows through a 6 KB LDS tile, summed per (graph, channel) in node order.
// Numerics: fp32; the online softmax reorders the rounding of the reference's two-pass softmax
// (tests/test_gpu_ops.py compares against the fp32 PyTorch reference at 2e-5).
#include <pybind11/pybind11.h>

#include "../common.h"

namespace py = pybind11;

namespace gsc {

constexpr int kNlMaxLayers = 16;
constexpr float kNlSlope = 0.2f;

struct NlArgs {
  const float* pparams;    // padded blocks: [Wl HP x FIP | bl HP | Wr HP x FIP | br HP | att HP | bias HP]
  const float* x;          // [B, P, Fin]
  const int32_t* topo;     // [B]
  const int32_t* in_src;   // [T, M] target-sorted messages: source node
  const int32_t* in_ptr;   // [T, P+1]
  const float* deg;        // [T, P]
  const int32_t* nnodes;   // [T]
  float* emb;              // [B, H]
  int B, P, Fin, H, L, M, NP, G;
  int layer_of[kNlMaxLayers];
};

template <int HP, int FIP>
__host__ __device__ constexpr int nl_block_floats() { return 2 * HP * FIP + 4 * HP; }

template <int HP>
__host__ __device__ inline long nl_block_offset(int b) {
  return b == 0 ? 0 : nl_block_floats<HP, 4>() + (long)(b - 1) * nl_block_floats<HP, HP>();
}

// Pad the module's parameter blocks (Wl [H,Fi], bl, Wr, br, att, bias) into HP x FIP tiles.
template <int HP>
__global__ void nl_pad_params_kernel(const float* __restrict__ src, float* __restrict__ dst, int n_blocks, int Fin,
                                     int H) {
  for (int b = blockIdx.x; b < n_blocks; b += gridDim.x) {
    const int Fi = b == 0 ? Fin : H;
    const int FIP = b == 0 ? 4 : HP;
    const float* s = src + (b == 0 ? 0 : (2 * H * Fin + 4 * H) + (long)(b - 1) * (2 * H * H + 4 * H));
    float* d = dst + nl_block_offset<HP>(b);
    const int nf = 2 * HP * FIP + 4 * HP;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) {
      float v = 0.f;
      const int WF = HP * FIP;
      if (i < WF) {                                   // Wl
        const int c = i / FIP, k = i % FIP;
        if (c < H && k < Fi) v = s[c * Fi + k];
      } else if (i < WF + HP) {                       // bl
        const int c = i - WF;
        if (c < H) v = s[H * Fi + c];
      } else if (i < 2 * WF + HP) {                   // Wr
        const int r = i - WF - HP, c = r / FIP, k = r % FIP;
        if (c < H && k < Fi) v = s[H * Fi + H + c * Fi + k];
      } else {                                        // br, att, bias
        const int r = i - 2 * WF - HP, which = r / HP, c = r % HP;
        if (c < H) v = s[2 * H * Fi + H + which * H + c];
      }
      d[i] = v;
    }
  }
}

template <int HP, int FIP>
__device__ __forceinline__ void nl_linear(const float* __restrict__ W, const float* __restrict__ bvec,
                                          const float (&h)[HP], float (&out)[HP]) {
#pragma unroll
  for (int c = 0; c < HP; ++c) {
    float s = bvec[c];
#pragma unroll
    for (int k = 0; k < FIP; ++k) s = fmaf(W[c * FIP + k], h[k], s);
    out[c] = s;
  }
}

// One convolution for the wave's node lanes; h (in, FIP valid entries) -> h (out, HP entries).
template <int HP, int FIP>
__device__ __forceinline__ void nl_conv(const float* __restrict__ blk, float (&h)[HP], int slot_base, bool valid,
                                        int q0, int deg_in, const int32_t* __restrict__ src, float inv_deg,
                                        int max_deg, bool relu) {
  const float* Wl = blk;
  const float* bl = Wl + HP * FIP;
  const float* Wr = bl + HP;
  const float* br = Wr + HP * FIP;
  const float* att = br + HP;
  const float* bias = att + HP;
  float xl[HP], xr[HP];
  nl_linear<HP, FIP>(Wl, bl, h, xl);
  nl_linear<HP, FIP>(Wr, br, h, xr);
  float acc[HP];
#pragma unroll
  for (int c = 0; c < HP; ++c) acc[c] = 0.f;
  float mx = -INFINITY, ssum = 0.f;
  for (int q = 0; q < max_deg; ++q) {          // wave-uniform trip count; lanes past their degree idle
    const bool act = valid && q < deg_in;
    const int j = act ? src[q0 + q] : 0;
    const int addr = (slot_base + j) << 2;
    float xj[HP];
#pragma unroll
    for (int c = 0; c < HP; ++c) xj[c] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(xl[c])));
    float e4[4] = {0.f, 0.f, 0.f, 0.f};  // four independent chains (the score is a 24-term dot product)
#pragma unroll
    for (int c = 0; c < HP; ++c) {
      const float z = xj[c] + xr[c];
      e4[c & 3] = fmaf(att[c], z > 0.f ? z : kNlSlope * z, e4[c & 3]);
    }
    const float e = (e4[0] + e4[1]) + (e4[2] + e4[3]);
    if (act) {
      const float mn = fmaxf(mx, e);
      const float sc = __expf(mx - mn);      // 0 on the first message (mx = -inf)
      const float p = __expf(e - mn);
      ssum = ssum * sc + p;
#pragma unroll
      for (int c = 0; c < HP; ++c) acc[c] = fmaf(p, xj[c], acc[c] * sc);
      mx = mn;
    }
  }
  const float norm = inv_deg / (ssum + 1e-16f);
#pragma unroll
  for (int c = 0; c < HP; ++c) {
    float o = fmaf(acc[c], norm, bias[c]);
    h[c] = relu ? fmaxf(o, 0.f) : o;
  }
}

template <int HP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void gnn_nl_fwd_kernel(NlArgs a) {
  __shared__ float pool[4][64][HP + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane / a.NP, v = lane - slot * a.NP;
  const int waves_total = gridDim.x * 4;
  for (long tile = (long)blockIdx.x * 4 + wave; tile * a.G < a.B; tile += waves_total) {
    const long g = tile * a.G + slot;
    const bool in_graph = slot < a.G && g < a.B;
    const int t = in_graph ? a.topo[g] : 0;
    const int n = a.nnodes[t];
    const bool valid = in_graph && v < n;
    const int32_t* ip = a.in_ptr + (long)t * (a.P + 1);
    const int q0 = valid ? ip[v] : 0;
    const int deg_in = valid ? ip[v + 1] - q0 : 0;
    const float inv_deg = valid ? 1.f / a.deg[(long)t * a.P + v] : 0.f;
    int max_deg = deg_in;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) max_deg = max(max_deg, __shfl_xor(max_deg, o));
    const int32_t* src = a.in_src + (long)t * a.M;
    float h[HP];
#pragma unroll
    for (int c = 0; c < HP; ++c) h[c] = 0.f;
    if (valid) {
      const float* xv = a.x + (g * a.P + v) * a.Fin;
      for (int k = 0; k < a.Fin && k < 4; ++k) h[k] = xv[k];
    }
    const int slot_base = slot * a.NP;
    for (int l = 0; l < a.L; ++l) {
      const bool relu = l < a.L - 1 || a.L == 1;
      const int b = a.layer_of[l];
      const float* blk = a.pparams + nl_block_offset<HP>(b);
      if (b == 0) nl_conv<HP, 4>(blk, h, slot_base, valid, q0, deg_in, src, inv_deg, max_deg, relu);
      else nl_conv<HP, HP>(blk, h, slot_base, valid, q0, deg_in, src, inv_deg, max_deg, relu);
    }
    // mean pool over the graph's nodes (node order, deterministic)
#pragma unroll
    for (int c = 0; c < HP; ++c) pool[wave][lane][c] = valid ? h[c] : 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int idx = lane; idx < a.G * a.H; idx += 64) {
      const int gs = idx / a.H, c = idx - gs * a.H;
      const long gg = tile * a.G + gs;
      if (gg < a.B) {
        const int nn = a.nnodes[a.topo[gg]];
        float s = 0.f;
        for (int u = 0; u < nn; ++u) s += pool[wave][gs * a.NP + u][c];
        a.emb[gg * a.H + c] = s / (float)nn;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------------------------------------
bool gnn_nl_supported(int Fin, int H, int NP, int L) { return Fin <= 4 && H <= 32 && NP >= 1 && NP <= 64 && L <= kNlMaxLayers; }

// args: mirrors of the GnnArgs fields this kernel needs; params = unpadded module layout
void gnn_nl_forward(const float* params, int n_blocks, const float* x, const int32_t* topo, const int32_t* in_src,
                    const int32_t* in_ptr, const float* deg, const int32_t* nnodes, float* emb, int B, int P, int Fin,
                    int H, int L, int M, int NP, const int* layer_of, uintptr_t stream, int cus) {
  static float* ws = nullptr;
  static size_t ws_floats = 0;
  const int HP = H <= 24 ? 24 : 32;
  const size_t need = (size_t)(2 * HP * 4 + 4 * HP) + (size_t)(n_blocks - 1) * (2 * HP * HP + 4 * HP);
  if (need > ws_floats) {  // grows only on the first call for a model (outside graph capture)
    if (ws) GSC_HIP_CHECK(hipFree(ws));
    GSC_HIP_CHECK(hipMalloc(&ws, need * sizeof(float)));
    ws_floats = need;
  }
  hipStream_t st = stream_of(stream);
  NlArgs a{};
  a.pparams = ws; a.x = x; a.topo = topo; a.in_src = in_src; a.in_ptr = in_ptr; a.deg = deg; a.nnodes = nnodes;
  a.emb = emb; a.B = B; a.P = P; a.Fin = Fin; a.H = H; a.L = L; a.M = M; a.NP = NP; a.G = 64 / NP;
  for (int i = 0; i < L; ++i) a.layer_of[i] = layer_of[i];
  const long tiles = (B + a.G - 1) / a.G;
  long grid = (tiles + 3) / 4;
  const long cap = (long)cus * 8;
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  if (HP == 24) {
    hipLaunchKernelGGL(nl_pad_params_kernel<24>, dim3(n_blocks), dim3(256), 0, st, params, ws, n_blocks, Fin, H);
    hipLaunchKernelGGL(gnn_nl_fwd_kernel<24>, dim3((unsigned)grid), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(nl_pad_params_kernel<32>, dim3(n_blocks), dim3(256), 0, st, params, ws, n_blocks, Fin, H);
    hipLaunchKernelGGL(gnn_nl_fwd_kernel<32>, dim3((unsigned)grid), dim3(256), 0, st, a);
  }
  check_launch();
}

}  // namespace gsc
