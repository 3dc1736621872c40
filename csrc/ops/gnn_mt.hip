// Multi-tile MFMA GATv2 embedder kernels (gfx950) for graphs of 33..64 nodes (BASELINE config 4:
// the 50-node gen_networks topologies): one graph per workgroup, one wave per 32-node tile.
//
// Wave w owns node rows [32w, 32w + 32) of every dense product and the messages whose TARGET lies
// in its tile (the message list is target-sorted, so that is one contiguous range per tile).  All
// products run on v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32 accumulation), as in gnn_mf.hip:
//
//   node linears      X_l, X_r = h W^T + b          row-local: own rows of h (LDS image)
//   aggregation       Y = E X_l + bias              A = E own rows, K = all nodes,
//                                                   B = X_l^T bf16 image (every tile's columns)
//   weight gradients  dW += dX^T h                  K = own nodes, straight from the accumulators
//   input gradients   dh = dX_l W_l + dX_r W_r      row-local
//   message scatter   dX_r = S_dst G                K = the tile's own messages
//                     dX_l = S_src G + E^T dy       K = all messages, then all nodes (dy^T image)
//
// Scores, the per-target softmax and the attention backward run per message on the VALU in fp32
// (PyG operation order); since a wave only touches messages INTO its own tile, the per-target
// max / sum atomics stay wave-local.  Cross-wave data (x_l rows, X_l^T, E^T, G^T, dy^T) is published
// with workgroup barriers: two per layer in each direction.  Double-buffered dy^T lets a wave write
// the next layer's gradient while its partner still reads this layer's.
//
// The grad-requiring forward saves each conv's input (bf16 rows + per-tile transposed image) and
// alpha to a per-graph HBM blob laid out per tile, so the backward loads exactly its own tile's
// bytes with direct global->LDS loads (no recompute of the forward, no cross-wave hazard on the
// staging buffer).
//
// Reference semantics: PyG GATv2Conv (/root/reference/src/rlsp/agents/models.py:10-53),
// gatv2_dense_reference in gsc_amd/models/gnn.py.  Tests: tests/test_gpu_ops.py (50-node graphs).
#include <pybind11/pybind11.h>

#include <cstdlib>

#include "gnn_mf.h"

namespace gsc {

constexpr int kMtTS = 40;  // bf16 row stride of the per-tile [k][32 nodes] images (80 B rows)

// Workgroup barrier ordering LDS only: the saved-state stores to HBM stay in flight across it (a
// plain __syncthreads() waits for every outstanding global store of the wave first)
__device__ __forceinline__ void mt_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct MtLayout {
  int NT, NV, NVS, MS;           // tiles, node rows (32 NT), bf16 stride of [.][node] images, G^T stride
  int hTrows0, hTrows;           // rows of the per-tile [k][node] images: encoder input (Fin -> 4), hidden
  // per-graph region (byte offsets)
  int xl, xr, xlT, E, sc, sm, topo, pool;  // forward (E doubles as E^T in the backward)
  int hR[2];                     // forward: ping-pong node images [NV][kMfRS] (save: h^T staged in dead rows)
  int ld, ldw;                   // backward: per-wave loaded layer images (own rows + own h^T), bytes per wave
  int al, da, dy, dyT[2], U, ss, wq; // backward
  int encW, encK;                // backward: per-wave encoder dW image
  int per_graph;                 // bytes of the per-graph region
  // saved blob per graph (HBM): per layer [tile chunk x NT][alpha]
  int blob, bl_layer[kClMaxLayers], bl_tile[kClMaxLayers];
};

__host__ __device__ __forceinline__ int mt_tile_hR_bytes() { return 32 * kMfRS * 2; }

// tile message range [q0, q1) (messages into nodes 32w .. 32w + 31) and the topology tables.  The
// topology (target-sorted message list, in-degrees) is cached per workgroup; every thread helps.
struct MtTopo {
  int *isrc, *idst;
  float* deg;
  int* iptr;  // [P + 1] message range of each target node (per-node softmax / sums without atomics)
  int n, m, t, q0, q1;
};

// The per-wave scalars (q0, q1, n, m) stay in registers while the topology does not change: a graph
// of the cached topology costs no dependent global round trip (its id is prefetched a graph ahead).
__device__ __forceinline__ void mt_load_topo(MtTopo& T, const ClArgs& a, int t, int w) {
  if (T.t == t) return;  // uniform over the workgroup: every wave holds the same T.t
  const int po = t * (a.P + 1);
  const int lo = 32 * w < a.P ? 32 * w : a.P, hi = 32 * w + 32 < a.P ? 32 * w + 32 : a.P;
  // wave-uniform: held in SGPRs (a VGPR holding a loaded value makes the compiler drain vmcnt -- and
  // with it the prefetches in flight -- in the preheader of every store loop that reads it)
  T.q0 = __builtin_amdgcn_readfirstlane(a.in_ptr[po + lo]);
  T.q1 = __builtin_amdgcn_readfirstlane(a.in_ptr[po + hi]);
  T.n = __builtin_amdgcn_readfirstlane(a.nnodes[t]);
  T.m = __builtin_amdgcn_readfirstlane(a.nmsgs[t]);
  T.t = t;
  const long mo = (long)t * a.M;
  // rows padded to MP with -1: the backward's one-hot operands (mt_onehot) read whole 16-message slices
  for (int i = threadIdx.x; i < a.MP; i += blockDim.x) {
    const bool v = i < T.m;
    T.isrc[i] = v ? a.in_src[mo + i] : -1;
    T.idst[i] = v ? a.in_dst[mo + i] : -1;
  }
  for (int i = threadIdx.x; i < a.P; i += blockDim.x) T.deg[i] = a.deg[(long)t * a.P + i];
  for (int i = threadIdx.x; i <= a.P; i += blockDim.x) T.iptr[i] = a.in_ptr[po + i];
}

// accumulator tile (rows = 32 nodes of the own tile, lane column c) -> bf16 [c][node] image at node
// column offset col0 (stride S); 4 consecutive rows per 8-byte store
__device__ __forceinline__ void mt_store_T(const f32x16& acc, __bf16* img, int S, int col0, int rows, int lane,
                                           bool relu) {
  const int r = lane & 31, hh = lane >> 5;
  if (r >= rows) return;
  __bf16* tb = img + r * S + col0 + 4 * hh;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bf16x4 t;
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = (__bf16)(relu ? fmaxf(acc[4 * g + j], 0.f) : acc[4 * g + j]);
    *reinterpret_cast<bf16x4*>(tb + 8 * g) = t;
  }
}

// One-hot MFMA A operand of the message matrices, generated from the LDS topology instead of loaded
// from the [T, NV, MP] bf16 tables in HBM: lane (row node, k half) gets 8 consecutive messages
// p[0..7] (16-B aligned, padded with -1 past the graph's messages) -> bf16 1.0 where p[j] == node.
// (A global fragment per MFMA step left every step waiting on an L2 round trip.)
__device__ __forceinline__ bf16x8 mt_onehot(const int* p, int node) {
  const int4 a = *reinterpret_cast<const int4*>(p);
  const int4 b = *reinterpret_cast<const int4*>(p + 4);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  u32x4 o;
  o[0] = (a.x == node ? 0x3F80u : 0u) | (a.y == node ? 0x3F800000u : 0u);
  o[1] = (a.z == node ? 0x3F80u : 0u) | (a.w == node ? 0x3F800000u : 0u);
  o[2] = (b.x == node ? 0x3F80u : 0u) | (b.y == node ? 0x3F800000u : 0u);
  o[3] = (b.z == node ? 0x3F80u : 0u) | (b.w == node ? 0x3F800000u : 0u);
  return __builtin_bit_cast(bf16x8, o);
}

// Input rows of the own tile held in registers a graph ahead (Fin <= 8: 32 Fin <= 256 floats, four per
// lane): loads at clamped addresses inside graph g's P rows, issued while the previous graph computes.
__device__ __forceinline__ bool mt_x_fits(const ClArgs& a) { return 32 * a.Fin <= 256; }
__device__ __forceinline__ void mt_x_prefetch(float (&xv)[4], const ClArgs& a, int g, int w, int lane) {
  const int rows = a.P - 32 * w, lim = (rows < 32 ? rows : 32) * a.Fin;
  const float* xg = a.x + ((long)g * a.P + 32 * w) * a.Fin;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = lane + 64 * u;
    xv[u] = xg[idx < lim ? idx : 0];
  }
}
// prefetched rows -> cleared bf16 row image (+ the transposed image), the nv real rows only
template <bool SAVE_T>
__device__ __forceinline__ void mt_x_scatter(const float (&xv)[4], int nv, int Fin, __bf16* hR, __bf16* hT, int TS,
                                             int trows, int lane) {
  for (int i = lane; i < 32 * 32; i += 64) {
    const int v = i >> 5, k = i & 31;
    hR[v * kMfRS + k] = (__bf16)0.f;
    if (SAVE_T && k < trows) hT[k * TS + v] = (__bf16)0.f;
  }
  const int nx = nv > 0 ? nv * Fin : 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = lane + 64 * u;
    if (idx < nx) {
      const int v = idx / Fin, k = idx - v * Fin;
      const __bf16 b = (__bf16)xv[u];
      hR[v * kMfRS + k] = b;
      if (SAVE_T) hT[k * TS + v] = b;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
template <int HPF, bool K2, bool SAVE>
__global__ __launch_bounds__(128) void gnn_mt_fwd_kernel(ClArgs a, MtLayout m) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, w = tid >> 6;
  mf_stage_vec(a, lds);
  const bf16x8* frags = reinterpret_cast<const bf16x8*>(lds + mf_vec_floats(a.n_blocks));
  mf_stage_frags(a, reinterpret_cast<bf16x8*>(lds + mf_vec_floats(a.n_blocks)), 2);
  char* const G = reinterpret_cast<char*>(lds + mf_vec_floats(a.n_blocks) + 2 * kMfFragSet);
  MtTopo T;
  T.isrc = reinterpret_cast<int*>(G + m.topo);
  T.idst = T.isrc + a.MP;
  T.deg = reinterpret_cast<float*>(T.idst + a.MP);
  T.iptr = reinterpret_cast<int*>(T.deg + a.P);
  T.t = -1;
  float* const xl = reinterpret_cast<float*>(G + m.xl);
  float* const xr = reinterpret_cast<float*>(G + m.xr);
  __bf16* const xlT = reinterpret_cast<__bf16*>(G + m.xlT);
  __bf16* const E = reinterpret_cast<__bf16*>(G + m.E);
  float* const sc = reinterpret_cast<float*>(G + m.sc);
  float* const sm = reinterpret_cast<float*>(G + m.sm);
  float* const pool = reinterpret_cast<float*>(G + m.pool);
  __syncthreads();
  // graph g + gridDim.x's topology id and input rows are loaded while graph g computes
  // a.work: graphs claimed from a zeroed counter by a full-device grid (as in the backward)
  int* const wq = reinterpret_cast<int*>(G + m.wq);
  int g = blockIdx.x, gq = blockIdx.x + gridDim.x;
  if (a.work) {
    if (tid == 0) {
      wq[0] = atomicAdd(a.work, 1);
      wq[1] = atomicAdd(a.work, 1);
    }
    __syncthreads();
    g = __builtin_amdgcn_readfirstlane(wq[0]);
    gq = __builtin_amdgcn_readfirstlane(wq[1]);
  }
  int claim = 0;
  bool first = true;
  const bool xpre = mt_x_fits(a);
  int t_cur = __builtin_amdgcn_readfirstlane(a.topo[g < a.B ? g : 0]);
  float xv[4];
  if (xpre) mt_x_prefetch(xv, a, g < a.B ? g : 0, w, tid & 63);
  while (g < a.B) {  // uniform over the workgroup
    const int lane = mf_lane(), r = lane & 31, hh = lane >> 5;
    if (!a.work) gq = g + gridDim.x;
    else if (!first) gq = __builtin_amdgcn_readfirstlane(wq[0]);  // published before the last graph's pool barrier
    first = false;
    const int gn = gq < a.B ? gq : g;
    mt_load_topo(T, a, __builtin_amdgcn_readfirstlane(t_cur), w);
    const int n = T.n, nl = n - 32 * w;  // real rows of the own tile (may be <= 0)
    // own rows: clear E, input features -> bf16 rows (and the saved per-tile transposed image)
    // save staging of the per-tile transposed image h^T (HPF x kMtTS bf16 <= one tile's 32 x kMfRS
    // rows): the own rows of the ping-pong buffer that holds nothing live -- hR[1] before layer 0, the
    // current layer's input (read only by its node linears) in each layer's epilogue.  No extra LDS, so
    // the saving forward keeps the plain forward's three workgroups per CU (was two at +3.8 KB).
    {
      __bf16* hA = reinterpret_cast<__bf16*>(G + m.hR[0]) + 32 * w * kMfRS;
      __bf16* hT = reinterpret_cast<__bf16*>(G + m.hR[1]) + 32 * w * kMfRS;
      if (xpre) {
        mt_x_scatter<SAVE>(xv, nl < 32 ? nl : 32, a.Fin, hA, hT, kMtTS, m.hTrows0, lane);
        t_cur = a.topo[gn];  // made uniform where it is used: a readfirstlane here would wait for it
        mt_x_prefetch(xv, a, gn, w, lane);
        if (a.work && tid == 0) claim = atomicAdd(a.work, 1);  // the graph after next
      } else {
        mf_stage_input<SAVE>(a.x + ((long)g * a.P + 32 * w) * a.Fin, nl < 32 ? nl : 32, a.Fin, 32, hA, hT, kMtTS,
                             m.hTrows0, lane);
        t_cur = a.topo[gn];
        if (a.work && tid == 0) claim = atomicAdd(a.work, 1);
      }
      uint4* e4 = reinterpret_cast<uint4*>(E + 32 * w * m.NVS);
      for (int i = lane; i < 32 * m.NVS / 8; i += 64) e4[i] = make_uint4(0, 0, 0, 0);
    }
    cl_wave_sync();
    if (SAVE) {  // layer-0 input chunk of the own tile
      char* dst = reinterpret_cast<char*>(a.blob) + (long)g * m.blob + m.bl_layer[0] + w * m.bl_tile[0];
      const uint4* s0 = reinterpret_cast<const uint4*>(G + m.hR[0] + 32 * w * kMfRS * 2);
      const uint4* s1 = reinterpret_cast<const uint4*>(G + m.hR[1] + 32 * w * kMfRS * 2);
      const int n0 = mt_tile_hR_bytes() / 16, n1 = m.hTrows0 * kMtTS * 2 / 16;
      for (int i = lane; i < n0 + n1; i += 64)
        reinterpret_cast<uint4*>(dst)[i] = i < n0 ? s0[i] : s1[i - n0];
    }
    mt_barrier();  // topology visible to every wave
    int cur = 0;
    float pl = 0.f;
    for (int l = 0; l < a.L; ++l) {
      const int lane = mf_lane(), r = lane & 31, hh = lane >> 5;
      const float* vec = lds + (l == 0 ? 0 : kMfVec);
      const __bf16* hin = reinterpret_cast<const __bf16*>(G + m.hR[cur]) + 32 * w * kMfRS;
      f32x16 al, ar;
      if (l == 0) mf_linear<false>(mf_frags(frags, 0, lane), vec, hin, 32, lane, al, ar);
      else mf_linear<K2>(mf_frags(frags, 1, lane), vec, hin, 32, lane, al, ar);
      mf_store_rows<HPF>(al, nl, xl + 32 * w * mf_xs(HPF), lane);
      mf_store_rows<HPF>(ar, nl, xr + 32 * w * mf_xs(HPF), lane);
      mt_store_T(al, xlT, m.NVS, 32 * w, HPF, lane, false);
      mt_barrier();  // B1: x_l rows and X_l^T of every tile
      // scores / softmax over the messages into the own tile (wave-local atomics)
      asm volatile("" ::: "memory");
      for (int q = T.q0 + lane; q < T.q1; q += 64) {
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
        sc[q] = s;
      }
      cl_wave_sync();
      // per-target max and exp-sum, lane = target node of the own tile over its contiguous message range
      // (the target-sorted list): no LDS atomics -- messages of one target sat in consecutive lanes, so
      // each atomic was an in-degree-way bank conflict
      if (lane < 32) {
        const int v = 32 * w + lane;
        float sum = 0.f;
        if (v < n) {
          const int qa = T.iptr[v], qb = T.iptr[v + 1];
          float mv = -INFINITY;
          for (int q = qa; q < qb; ++q) mv = fmaxf(mv, sc[q]);
          for (int q = qa; q < qb; ++q) {
            const float ex = __expf(sc[q] - mv);
            sc[q] = ex;
            sum += ex;
          }
        }
        sm[v] = sum;
      }
      cl_wave_sync();
      for (int q = T.q0 + lane; q < T.q1; q += 64) {
        const int i = T.idst[q];
        const float al_q = sc[q] / (sm[i] + 1e-16f);
        sc[q] = al_q;
        E[i * m.NVS + T.isrc[q]] = (__bf16)(al_q / T.deg[i]);
        if (SAVE)
          reinterpret_cast<float*>(reinterpret_cast<char*>(a.blob) + (long)g * m.blob + m.bl_layer[l] +
                                   m.NT * m.bl_tile[l])[q] = al_q;
      }
      cl_wave_sync();
      // Y = E X_l + bias (own rows, K = every node)
      f32x16 y;
      {
        const float bc = vec[96 + r];
#pragma unroll
        for (int i = 0; i < 16; ++i) y[i] = bc;
        const __bf16* erow = E + (32 * w + r) * m.NVS + 8 * hh;
        const __bf16* xrow = xlT + (r < HPF ? r : 0) * m.NVS + 8 * hh;
        for (int s = 0; 16 * s < n; ++s)
          y = mf_mma(*reinterpret_cast<const bf16x8*>(erow + 16 * s), *reinterpret_cast<const bf16x8*>(xrow + 16 * s), y);
      }
      const int nn = nl - 4 * hh;
      if (l + 1 == a.L) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) < nn) pl += y[i];
      } else {
        __bf16* hb = reinterpret_cast<__bf16*>(G + m.hR[cur ^ 1]) + 32 * w * kMfRS + 4 * hh * kMfRS + r;
        f32x16 o;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o[i] = ((i & 3) + 8 * (i >> 2) < nn && r < a.H) ? fmaxf(y[i], 0.f) : 0.f;
          hb[((i & 3) + 8 * (i >> 2)) * kMfRS] = (__bf16)o[i];
        }
        if (SAVE) {
          __bf16* hT = reinterpret_cast<__bf16*>(G + m.hR[cur]) + 32 * w * kMfRS;  // dead input rows
          mt_store_T(o, hT, kMtTS, 0, HPF, lane, false);
          cl_wave_sync();
          char* dst = reinterpret_cast<char*>(a.blob) + (long)g * m.blob + m.bl_layer[l + 1] + w * m.bl_tile[l + 1];
          const uint4* s0 = reinterpret_cast<const uint4*>(G + m.hR[cur ^ 1] + 32 * w * kMfRS * 2);
          const uint4* s1 = reinterpret_cast<const uint4*>(G + m.hR[cur] + 32 * w * kMfRS * 2);
          const int n0 = mt_tile_hR_bytes() / 16, n1 = m.hTrows * kMtTS * 2 / 16;
          for (int i = lane; i < n0 + n1; i += 64)
            reinterpret_cast<uint4*>(dst)[i] = i < n0 ? s0[i] : s1[i - n0];
        }
        cur ^= 1;
      }
      mt_barrier();  // B2: every wave is done with this layer's x_l / X_l^T
    }
    {
      const int lane = mf_lane(), c = lane & 31, hh = lane >> 5;
      pl += __shfl_xor(pl, 32);
      if (hh == 0) pool[32 * w + c] = pl;
      if (a.work && tid == 0) wq[0] = claim;
      mt_barrier();
      if (w == 0 && hh == 0 && c < a.H) {
        float s = 0.f;
        for (int t2 = 0; t2 < m.NT; ++t2) s += pool[32 * t2 + c];
        a.emb[(long)g * a.H + c] = s / (float)n;
      }
    }
    g = gq;
  }
}

// ---------------------------------------------------------------------------------------------
// backward (loads the forward's saved per-tile state)
// ---------------------------------------------------------------------------------------------
// attention backward of the own messages, lane = (message, quarter of the channels)
template <int HPF>
__device__ __forceinline__ void mt_att_bwd(const MtTopo& T, const float* da, const float* al, const float* ssum,
                                           const float* xl, const float* xr, const float* vec, __bf16* U, int MS,
                                           int lane, float (&gatt)[HPF / 4]) {
  constexpr int CG = HPF / 4;
  const int grp = lane & 3, c0 = grp * CG;
  for (int q = T.q0 + (lane >> 2); q < T.q1; q += 16) {
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
}

// issue (do not wait for) graph g's saved state of layer l: the own-tile images into this wave's ld
// region and alpha of the own messages (16-B aligned superset) into the shared alpha region
__device__ __forceinline__ void mt_issue_saved(const ClArgs& a, const MtLayout& m, const MtTopo& T, char* G, int g,
                                               int l, int w, int lane) {
  const char* src = reinterpret_cast<const char*>(a.blob) + (long)g * m.blob + m.bl_layer[l];
  const char* st = src + w * m.bl_tile[l];
  char* const ld = G + m.ld + w * m.ldw;
  const int tb = m.bl_tile[l];
  for (int o = 0; o < tb; o += 1024)
    if (o + 16 * lane < tb)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(st + o + 16 * lane),
                                       (__attribute__((address_space(3))) void*)(ld + o), 16, 0, 0);
  const int a0 = (T.q0 & ~3) * 4, a1 = ((T.q1 + 3) & ~3) * 4;
  const char* sa = src + m.NT * tb;
  for (int o = a0; o < a1; o += 1024)
    if (o + 16 * lane < a1)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(sa + o + 16 * lane),
                                       (__attribute__((address_space(3))) void*)(G + m.al + o), 16, 0, 0);
}

template <int HPF, bool K2>
__global__ __launch_bounds__(128) void gnn_mt_bwd_kernel(ClArgs a, MtLayout m) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int CG = HPF / 4;
  const int tid = threadIdx.x, w = tid >> 6;
  mf_stage_vec(a, lds);
  const bf16x8* frags = reinterpret_cast<const bf16x8*>(lds + mf_vec_floats(a.n_blocks));
  mf_stage_frags(a, reinterpret_cast<bf16x8*>(lds + mf_vec_floats(a.n_blocks)), 3);
  char* const G = reinterpret_cast<char*>(lds + mf_vec_floats(a.n_blocks) + 3 * kMfFragSet);
  MtTopo T;
  T.isrc = reinterpret_cast<int*>(G + m.topo);
  T.idst = T.isrc + a.MP;
  T.deg = reinterpret_cast<float*>(T.idst + a.MP);
  T.iptr = reinterpret_cast<int*>(T.deg + a.P);
  T.t = -1;
  {
    const int lane = tid & 63;
    // G^T columns beyond a graph's messages meet zeros of S but must be finite; E^T starts clear
    for (int i = tid; i < HPF * m.MS / 8; i += blockDim.x) reinterpret_cast<uint4*>(G + m.U)[i] = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < m.NV * m.NVS / 8; i += blockDim.x) reinterpret_cast<uint4*>(G + m.E)[i] = make_uint4(0, 0, 0, 0);
    float* encW = reinterpret_cast<float*>(G + m.encW) + w * 2 * 32 * m.encK;
    for (int i = lane; i < 2 * 32 * m.encK; i += 64) encW[i] = 0.f;
  }
  __syncthreads();
  f32x16 gPl, gPr;
  mf_zero(gPl);
  mf_zero(gPr);
  MfVecGrad GE{0.f, 0.f, 0.f}, GP{0.f, 0.f, 0.f};
  float gattE[CG], gattP[CG];
#pragma unroll
  for (int k = 0; k < CG; ++k) gattE[k] = gattP[k] = 0.f;
  const int NVS = m.NVS, MS = m.MS;
  // Software pipeline over the graph loop: the next graph's topology id and d emb row are loaded during
  // this graph's first processed conv, and each conv's saved state (plus, for a graph of the cached
  // topology, the next graph's first one) is issued at the end of the conv before it: the loads whose
  // round trips the one wave per SIMD used to wait out in full.
  //
  // With a.work (overlap mode: the grid covers every CU, including the simulator's, whose LDS frees up
  // when its kernel ends) graphs are claimed from a zeroed counter instead of a fixed stride: workgroups
  // placed late take what is left instead of a fixed share.  Wave 0 lane 0 claims the graph after next
  // during the first conv (its round trip overlaps the conv) and publishes it in LDS for the next graph.
  int* const wq = reinterpret_cast<int*>(G + m.wq);
  int g = blockIdx.x, gq = blockIdx.x + gridDim.x;
  if (a.work) {
    if (tid == 0) {
      wq[0] = atomicAdd(a.work, 1);
      wq[1] = atomicAdd(a.work, 1);
    }
    __syncthreads();
    g = __builtin_amdgcn_readfirstlane(wq[0]);
    gq = __builtin_amdgcn_readfirstlane(wq[1]);
  }
  int claim = 0;
  bool first = true;
  int t_cur = __builtin_amdgcn_readfirstlane(a.topo[g < a.B ? g : 0]), t_next = t_cur;
  float ge_cur = a.demb[(long)(g < a.B ? g : 0) * a.H + ((tid & 31) < a.H ? (tid & 31) : 0)];
  float ge_next = ge_cur;
  bool pre = false;  // this graph's first processed conv's saved state is already in flight
  while (g < a.B) {  // uniform over the workgroup
    // the partner may still read dy^T / E^T / the topology of the previous graph's first conv
    mt_barrier();
    int lane = mf_lane();
    if (!a.work) gq = g + gridDim.x;
    else if (!first) gq = __builtin_amdgcn_readfirstlane(wq[0]);  // written by wave 0 before the barrier
    first = false;
    const bool has_next = gq < a.B;
    const int gn = has_next ? gq : g;
    mt_load_topo(T, a, __builtin_amdgcn_readfirstlane(t_cur), w);
    const int n = T.n, nl = n - 32 * w;
    float* const xl = reinterpret_cast<float*>(G + m.xl);
    float* const xr = reinterpret_cast<float*>(G + m.xr);
    float* const dy = reinterpret_cast<float*>(G + m.dy);
    float* const da = reinterpret_cast<float*>(G + m.da);
    float* const al = reinterpret_cast<float*>(G + m.al);
    float* const ssum = reinterpret_cast<float*>(G + m.ss);
    __bf16* const ET = reinterpret_cast<__bf16*>(G + m.E);
    __bf16* const U = reinterpret_cast<__bf16*>(G + m.U);
    char* const ld = G + m.ld + w * m.ldw;
    // d emb -> dy of the last conv (mean pool; the last conv has no ReLU): tile, fp32 rows, dy^T
    f32x16 dyt;
    {
      const int c = lane & 31, hh = lane >> 5;
      const float ge = c < a.H ? ge_cur / (float)n : 0.f;
      const int nn = nl - 4 * hh;
#pragma unroll
      for (int i = 0; i < 16; ++i) dyt[i] = (i & 3) + 8 * (i >> 2) < nn ? ge : 0.f;
      mf_store_rows<HPF>(dyt, nl, dy + 32 * w * mf_xs(HPF), lane);
      mt_store_T(dyt, reinterpret_cast<__bf16*>(G + m.dyT[(a.L - 1) & 1]), NVS, 32 * w, HPF, lane, false);
    }
    for (int l = a.L - 1; l >= 0; --l) {
      lane = mf_lane();
      const int r = lane & 31, hh = lane >> 5;
      const float* vec = lds + (l == 0 ? 0 : kMfVec);
      const int hrows = l == 0 ? m.hTrows0 : m.hTrows;
      // this layer's saved own-tile images (rows of h, per-tile h^T) and alpha of the own messages
      if (!pre) mt_issue_saved(a, m, T, G, g, l, w, lane);
      pre = false;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cl_wave_sync();
      if (l == a.L - 1) {  // the next graph's scalars ride along with this conv
        t_next = a.topo[gn];  // made uniform where it is used
        ge_next = a.demb[(long)gn * a.H + (r < a.H ? r : 0)];
        if (a.work && tid == 0) claim = atomicAdd(a.work, 1);  // the graph after next
      }
      const __bf16* hin = reinterpret_cast<const __bf16*>(ld);                  // [32][kMfRS]
      const __bf16* hT = reinterpret_cast<const __bf16*>(ld + mt_tile_hR_bytes());  // [hrows][kMtTS]
      {
        f32x16 xa, xb;
        if (l == 0) mf_linear<false>(mf_frags(frags, 0, lane), vec, hin, 32, lane, xa, xb);
        else mf_linear<K2>(mf_frags(frags, 1, lane), vec, hin, 32, lane, xa, xb);
        mf_store_rows<HPF>(xa, nl, xl + 32 * w * mf_xs(HPF), lane);
        mf_store_rows<HPF>(xb, nl, xr + 32 * w * mf_xs(HPF), lane);
      }
      mt_barrier();  // B1: x_l rows, dy^T of every tile; E^T rows cleared
      // p_q = alpha_q (dy[i] . x_l[j]) / deg_i ; ssum_i = sum_{q -> i} p_q ; E^T[j][i] = alpha_q / deg_i
      asm volatile("" ::: "memory");
      for (int q = T.q0 + lane; q < T.q1; q += 64) {
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
        ET[j * NVS + i] = (__bf16)ad;
      }
      cl_wave_sync();
      // ssum_i per target node over its contiguous message range (no LDS atomics)
      if (lane < 32) {
        const int v = 32 * w + lane;
        float sum = 0.f;
        if (v < n)
          for (int q = T.iptr[v]; q < T.iptr[v + 1]; ++q) sum += da[q];
        ssum[v] = sum;
      }
      cl_wave_sync();
      // de_q = p_q - alpha_q ssum_i ; per channel z = x_l[j] + x_r[i]:
      //   d att_c += de_q lrelu(z) ;  G[q][c] = de_q att_c lrelu'(z)   (stored as G^T[c][q], bf16)
      if (l == 0) mt_att_bwd<HPF>(T, da, al, ssum, xl, xr, vec, U, MS, lane, gattE);
      else mt_att_bwd<HPF>(T, da, al, ssum, xl, xr, vec, U, MS, lane, gattP);
      mt_barrier();  // B2: E^T and G^T of every tile
      const int nn = nl - 4 * hh;
      if (l == 0) GE.bias += mf_colsum(dyt, nn);
      else GP.bias += mf_colsum(dyt, nn);
      f32x16 dxl, dxr;
      mf_zero(dxl);
      mf_zero(dxr);
      {
        const int node = 32 * w + r;
        const __bf16* gb = U + (r < HPF ? r : 0) * MS + 8 * hh;  // channels >= HPF: any finite data
        // dX_r: rows of S_dst are zero outside the own messages
        for (int s = T.q0 >> 4; 16 * s < T.q1; ++s)
          dxr = mf_mma(mt_onehot(T.idst + 16 * s + 8 * hh, node), *reinterpret_cast<const bf16x8*>(gb + 16 * s), dxr);
        for (int s = 0; 16 * s < T.m; ++s)
          dxl = mf_mma(mt_onehot(T.isrc + 16 * s + 8 * hh, node), *reinterpret_cast<const bf16x8*>(gb + 16 * s), dxl);
        const __bf16* erow = ET + (32 * w + r) * NVS + 8 * hh;
        const __bf16* yrow = reinterpret_cast<const __bf16*>(G + m.dyT[l & 1]) + (r < HPF ? r : 0) * NVS + 8 * hh;
        for (int s = 0; 16 * s < n; ++s)
          dxl = mf_mma(*reinterpret_cast<const bf16x8*>(erow + 16 * s), *reinterpret_cast<const bf16x8*>(yrow + 16 * s), dxl);
      }
      if (l == 0) {
        GE.bl += mf_colsum(dxl, nn);
        GE.br += mf_colsum(dxr, nn);
      } else {
        GP.bl += mf_colsum(dxl, nn);
        GP.br += mf_colsum(dxr, nn);
      }
      // dW[c][k] += sum_v dX[v][c] h[v][k] over the own nodes: dX^T from the accumulators
      f32x16 gEl, gEr;
      if (l == 0) {
        mf_zero(gEl);
        mf_zero(gEr);
      }
      {
        const __bf16* hrow = hT + (r < hrows ? r : 0) * kMtTS;  // columns k >= hrows of dW are discarded
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 hb = mf_perm_frag(hrow, s, hh);
          if (l == 0) {
            gEl = mf_mma(mf_pack(dxl, s), hb, gEl);
            gEr = mf_mma(mf_pack(dxr, s), hb, gEr);
          } else {
            gPl = mf_mma(mf_pack(dxl, s), hb, gPl);
            gPr = mf_mma(mf_pack(dxr, s), hb, gPr);
          }
        }
      }
      __bf16* const etw = ET + 32 * w * NVS;  // own rows of E^T: free once read above
      if (l > 0) {
        // dh = dX_l W_l + dX_r W_r (own rows): dX as bf16 row images in the own E^T rows
        __bf16* xlR = etw;
        __bf16* xrR = etw + 32 * kMfRS;
        {
          __bf16* bl = xlR + 4 * hh * kMfRS + r;
          __bf16* br = xrR + 4 * hh * kMfRS + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ro = (i & 3) + 8 * (i >> 2);
            bl[ro * kMfRS] = (__bf16)dxl[i];
            br[ro * kMfRS] = (__bf16)dxr[i];
          }
        }
        cl_wave_sync();
        asm volatile("" ::: "memory");
        const MfW wT = mf_frags(frags, 2, lane);
        f32x16 acc;
        mf_zero(acc);
        acc = mf_mma(*reinterpret_cast<const bf16x8*>(xlR + r * kMfRS + 8 * hh), wT.l[0], acc);
        acc = mf_mma(*reinterpret_cast<const bf16x8*>(xrR + r * kMfRS + 8 * hh), wT.r[0], acc);
        if (K2) {
          acc = mf_mma(*reinterpret_cast<const bf16x8*>(xlR + r * kMfRS + 16 + 8 * hh), wT.l[1], acc);
          acc = mf_mma(*reinterpret_cast<const bf16x8*>(xrR + r * kMfRS + 16 + 8 * hh), wT.r[1], acc);
        }
        // ReLU mask of this conv's input (the previous conv's output)
        const __bf16* mb = hin + 4 * hh * kMfRS + r;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int ro = (i & 3) + 8 * (i >> 2);
          dyt[i] = (ro < nn && (float)mb[ro * kMfRS] > 0.f) ? acc[i] : 0.f;
        }
        mf_store_rows<HPF>(dyt, nl, dy + 32 * w * mf_xs(HPF), lane);
        mt_store_T(dyt, reinterpret_cast<__bf16*>(G + m.dyT[(l - 1) & 1]), NVS, 32 * w, HPF, lane, false);
        cl_wave_sync();
      } else {
        // encoder dW (k < Fin columns) -> per-wave LDS image
        if (r < a.Fin) {
          float* el = reinterpret_cast<float*>(G + m.encW) + w * 2 * 32 * m.encK + 4 * hh * m.encK + r;
          float* er = el + 32 * m.encK;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ro = (i & 3) + 8 * (i >> 2);
            el[ro * m.encK] += gEl[i];
            er[ro * m.encK] += gEr[i];
          }
        }
      }
      // clear the own E^T rows for the next layer's scatter (other waves write them only after B1)
      for (int i = lane; i < 32 * NVS / 8; i += 64) reinterpret_cast<uint4*>(etw)[i] = make_uint4(0, 0, 0, 0);
      cl_wave_sync();
      // the next conv's saved state: this wave's ld images are dead (dW / dh / ReLU mask read above) and
      // both waves are past B2, the last read of the shared alpha region.  Issued after the last LDS
      // access of the conv: the compiler makes any later LDS access wait for LDS-DMA loads.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (l > 0) {
        mt_issue_saved(a, m, T, G, g, l - 1, w, lane);
        pre = true;
      } else if (has_next && __builtin_amdgcn_readfirstlane(t_next) == T.t) {
        mt_issue_saved(a, m, T, G, gn, a.L - 1, w, lane);
        pre = true;
      }
    }
    t_cur = t_next;
    ge_cur = ge_next;
    if (a.work && tid == 0) wq[0] = claim;  // read by both waves after the next graph's first barrier
    g = gq;
  }
  // per-wave gradients -> LDS images (the whole per-graph region is free now) -> workgroup sum
  __syncthreads();
  const int lane = tid & 63, r = lane & 31, hh = lane >> 5, c = r;
  float* img = reinterpret_cast<float*>(G) + w * kMfFlush;
  const int off1 = cl_block_offset(1, a.Fin, a.H);
  for (int b = 0; b < 2; ++b) {
    __syncthreads();
    if (b == 0) {
      const float* ew = reinterpret_cast<const float*>(G + m.encW) + w * 2 * 32 * m.encK;
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
    const MfVecGrad& VG = b == 0 ? GE : GP;
    const float bl = VG.bl + __shfl_xor(VG.bl, 32), br = VG.br + __shfl_xor(VG.br, 32);
    const float bi = VG.bias + __shfl_xor(VG.bias, 32);
    float* v = img + 2 * 32 * 32;
    if (hh == 0) { v[c] = bl; v[32 + c] = br; v[96 + c] = bi; }
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
      for (int t2 = 0; t2 < m.NT; ++t2) s += reinterpret_cast<const float*>(G)[t2 * kMfFlush + idx];
      a.partials[(long)blockIdx.x * a.n_params + first + rr] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
enum { kMtFwd = 0, kMtSave = 1, kMtBwd = 2 };
static MtLayout mt_layout(const ClArgs& a, int kind, int HPF) {
  MtLayout m{};
  m.NT = (a.NM + 31) / 32;
  m.NV = 32 * m.NT;
  // 16-B aligned rows; own-tile rows of E^T (32 x NVS) hold the two dX row images (NVS >= 80).  The row
  // stride in 16-B units must be odd: the MFMA operand reads (ds_read_b128, lane r = row r) then hit 16
  // distinct bank quads per lane group (NV 64: 88, not 80 -- 80 B-quads mod 64 banks repeat every 8 rows)
  m.NVS = m.NV + 16;
  if (((m.NVS / 8) & 1) == 0) m.NVS += 8;
  m.MS = a.MP + 8;
  m.hTrows0 = (a.Fin + 3) & ~3;
  m.hTrows = HPF;
  // saved blob: per layer NT tile chunks (h rows, h^T) + alpha
  int b = 0;
  for (int l = 0; l < a.L; ++l) {
    m.bl_layer[l] = b;
    m.bl_tile[l] = mt_tile_hR_bytes() + (l == 0 ? m.hTrows0 : m.hTrows) * kMtTS * 2;
    b += m.NT * m.bl_tile[l] + ((a.M + 3) & ~3) * 4;
  }
  m.blob = (b + 15) & ~15;
  int o = 0;
  auto take = [&](int bytes) {
    const int at = o;
    o += (bytes + 15) & ~15;
    return at;
  };
  // fp32 row images (x_l, x_r, dy) are read and written per message / per real node only: NM rows, not
  // NV (keeps the backward at two workgroups per CU with the wider NVS)
  const int fb = a.NM * mf_xs(HPF) * 4, M4b = ((a.M + 3) & ~3) * 4;
  m.xl = take(fb);
  m.xr = take(fb);
  m.E = take(m.NV * m.NVS * 2);
  m.topo = take((2 * a.MP + 2 * a.P + 1) * 4);
  if (kind != kMtBwd) {
    m.hR[0] = take(m.NV * kMfRS * 2);
    m.hR[1] = take(m.NV * kMfRS * 2);
    m.xlT = take(HPF * m.NVS * 2);
    m.sc = take(M4b);
    m.sm = take(m.NV * 4);
    m.pool = take(m.NT * 32 * 4);
    m.wq = take(16);  // work queue: the graph after next, claimed by wave 0 lane 0
    static_assert(32 * kMtTS <= 32 * kMfRS, "the h^T staging must fit one tile's rows of hR");
  } else {
    m.ldw = (mt_tile_hR_bytes() + HPF * kMtTS * 2 + 15) & ~15;
    m.ld = take(m.NT * m.ldw);
    m.al = take(M4b + 64);  // the 16-B aligned superset of each tile's message range
    m.da = take(M4b);
    m.dy = take(fb);
    m.dyT[0] = take(HPF * m.NVS * 2);
    m.dyT[1] = take(HPF * m.NVS * 2);
    m.U = take(HPF * m.MS * 2);
    m.ss = take(m.NV * 4);
    m.wq = take(16);  // work queue: the graph after next, claimed by wave 0 lane 0
    if (o < m.NT * kMfFlush * 4) o = m.NT * kMfFlush * 4;  // end-of-kernel per-wave gradient images
    m.encK = (a.Fin + 3) & ~3;
    m.encW = take(m.NT * 2 * 32 * m.encK * 4);  // beyond the end-of-kernel images
  }
  m.per_graph = (o + 15) & ~15;
  return m;
}

bool gnn_mt_supported(int Fin, int H, int NM, int M, int L, int n_blocks, const int* layer_of) {
  if (!(Fin <= 16 && H <= 32 && NM > 32 && NM <= 64 && L >= 2 && L <= kClMaxLayers && n_blocks == 2)) return false;
  for (int l = 0; l < L; ++l)
    if ((l == 0) != (layer_of[l] == 0)) return false;
  ClArgs a{};
  a.Fin = Fin; a.H = H; a.NM = NM; a.M = M; a.P = NM; a.MP = ((M + 15) / 16) * 16; a.L = L; a.n_blocks = n_blocks;
  const int HPF = H <= 24 ? 24 : 32;
  const MtLayout f = mt_layout(a, kMtSave, HPF), bw = mt_layout(a, kMtBwd, HPF);
  const size_t fl = sizeof(float) * (mf_vec_floats(2) + 2 * kMfFragSet) + (size_t)f.per_graph;
  const size_t bl = sizeof(float) * (mf_vec_floats(2) + 3 * kMfFragSet) + (size_t)bw.per_graph;
  return fl <= 160 * 1024 && bl <= 160 * 1024;
}

static size_t mt_lds(const ClArgs& a, const MtLayout& m, int sets) {
  return sizeof(float) * (mf_vec_floats(a.n_blocks) + sets * kMfFragSet) + (size_t)m.per_graph;
}

template <int HPF, bool K2>
static void mt_launch_fwd(ClArgs a, hipStream_t st, int cus) {
  const bool save = a.blob != nullptr;
  const MtLayout m = mt_layout(a, save ? kMtSave : kMtFwd, HPF);
  const size_t lds = mt_lds(a, m, 2);
  GSC_CHECK(lds <= 160 * 1024, "GNN (MFMA multi-tile) forward working set exceeds LDS");
  const void* fn = save ? (const void*)gnn_mt_fwd_kernel<HPF, K2, true> : (const void*)gnn_mt_fwd_kernel<HPF, K2, false>;
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu > 8) per_cu = 8;
  if (per_cu < 1) per_cu = 1;
  int grid = cus * per_cu;
  if (grid > a.B) grid = a.B;
  if (grid < 1) grid = 1;
  a.waves = m.NT;
  if (save)
    hipLaunchKernelGGL((gnn_mt_fwd_kernel<HPF, K2, true>), dim3(grid), dim3(64 * m.NT), lds, st, a, m);
  else
    hipLaunchKernelGGL((gnn_mt_fwd_kernel<HPF, K2, false>), dim3(grid), dim3(64 * m.NT), lds, st, a, m);
  check_launch();
}

template <int HPF, bool K2>
static int mt_launch_bwd(ClArgs a, hipStream_t st, int cus, int max_rows) {
  GSC_CHECK(a.MP >= a.M && a.MP % 16 == 0, "multi-tile MFMA GNN backward: message rows padded to 16");
  GSC_CHECK(a.blob != nullptr, "multi-tile MFMA GNN backward needs the forward's saved state");
  const MtLayout m = mt_layout(a, kMtBwd, HPF);
  const size_t lds = mt_lds(a, m, 3);
  GSC_CHECK(lds <= 160 * 1024, "GNN (MFMA multi-tile) backward working set exceeds LDS");
  const void* fn = (const void*)gnn_mt_bwd_kernel<HPF, K2>;
  if (lds > 65536) GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu > 8) per_cu = 8;
  if (per_cu < 1) per_cu = 1;
  int grid = cus * per_cu;
  if (grid > a.B) grid = a.B;
  if (grid > max_rows) grid = max_rows;
  if (grid < 1) grid = 1;
  a.waves = m.NT;
  hipLaunchKernelGGL((gnn_mt_bwd_kernel<HPF, K2>), dim3(grid), dim3(64 * m.NT), lds, st, a, m);
  check_launch();
  return grid;
}

void gnn_mt_forward(const void* args_generic, uintptr_t stream, int cus) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 16) mt_launch_fwd<24, false>(a, stream_of(stream), cus);
  else if (a.H <= 24) mt_launch_fwd<24, true>(a, stream_of(stream), cus);
  else mt_launch_fwd<32, true>(a, stream_of(stream), cus);
}

int gnn_mt_saved_bytes(const void* args_generic) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  return mt_layout(a, kMtBwd, a.H <= 24 ? 24 : 32).blob;
}

int gnn_mt_backward(const void* args_generic, uintptr_t stream, int cus, int max_rows) {
  const ClArgs& a = *reinterpret_cast<const ClArgs*>(args_generic);
  if (a.H <= 16) return mt_launch_bwd<24, false>(a, stream_of(stream), cus, max_rows);
  if (a.H <= 24) return mt_launch_bwd<24, true>(a, stream_of(stream), cus, max_rows);
  return mt_launch_bwd<32, true>(a, stream_of(stream), cus, max_rows);
}

}  // namespace gsc
