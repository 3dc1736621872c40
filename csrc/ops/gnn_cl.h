// Shared argument block and per-wave topology helpers of the fused GATv2 kernels
// (channel-lane gnn_cl.hip, MFMA gnn_mf.hip; dispatched from gnn.hip).
#pragma once
#include "../common.h"

namespace gsc {

constexpr int kClMaxLayers = 16;
constexpr float kClSlope = 0.2f;

// Optional per-phase cycle counters of the backward (s_memtime; gnn_cl_set_profile).
struct ClClock {
  unsigned long long last, acc[12];
  bool on;
  __device__ __forceinline__ void start(bool enable) {
    on = enable;
    for (int k = 0; k < 12; ++k) acc[k] = 0;
    if (on) last = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void mark(int k) {
    if (__builtin_constant_p(on) && !on) return;
    if (on) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
};

struct ClArgs {
  const float* params;     // unpadded module layout (Wl, bl, Wr, br, att, bias per block)
  const float* x;          // [B, P, Fin]
  const int32_t* topo;     // [B]
  const int32_t* in_src;   // [T, M]  messages sorted by target node: source
  const int32_t* in_dst;   // [T, M]  ... and target
  const int32_t* in_ptr;   // [T, P+1]
  const int32_t* out_q;    // [T, M]  messages sorted by source node: position in the target-sorted order
  const int32_t* out_ptr;  // [T, P+1]
  const int32_t* out_dst;  // [T, M]  ... and target
  const float* deg;
  const int32_t* nnodes;
  const int32_t* nmsgs;
  float* emb;              // [B, H]
  const float* demb;       // [B, H]
  float* partials;         // [grid, n_params] (unpadded layout)
  int B, P, Fin, H, L, M, NM, n_params, n_blocks, waves;
  int layer_of[kClMaxLayers];
  unsigned long long* prof;  // 12 phase counters or null
  const void* s_dst;         // MFMA backward: bf16 [T, 32, MP] one-hot target / source of each message
  const void* s_src;
  int MP;                    // messages padded to a multiple of 16
  void* blob;                // MFMA path: per-graph forward state saved for the backward (or null)
};

__device__ __forceinline__ void cl_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ __forceinline__ int cl_block_size(int Fi, int H) { return 2 * H * Fi + 4 * H; }
__host__ __device__ __forceinline__ int cl_block_offset(int b, int Fin, int H) {
  return b == 0 ? 0 : cl_block_size(Fin, H) + (b - 1) * cl_block_size(H, H);
}
struct ClTopo {
  int *isrc, *idst, *iptr, *oq, *odst, *optr;
  float* deg;
  int n, m, t;
};

__host__ __device__ __forceinline__ int cl_topo_ints(const ClArgs& a) { return ((4 * a.M + 2 * (a.P + 1) + a.P) + 3) & ~3; }

__device__ __forceinline__ void cl_bind_topo(ClTopo& T, int* base, const ClArgs& a) {
  T.isrc = base;
  T.idst = T.isrc + a.M;
  T.oq = T.idst + a.M;
  T.odst = T.oq + a.M;
  T.iptr = T.odst + a.M;
  T.optr = T.iptr + a.P + 1;
  T.deg = reinterpret_cast<float*>(T.optr + a.P + 1);
  T.t = -1;
}

__device__ __forceinline__ void cl_load_topo(ClTopo& T, const ClArgs& a, int t, int lane) {
  T.n = a.nnodes[t];
  T.m = a.nmsgs[t];
  if (T.t == t) return;
  T.t = t;
  const long mo = (long)t * a.M, po = (long)t * (a.P + 1);
  for (int i = lane; i < a.M; i += 64) {
    T.isrc[i] = a.in_src[mo + i];
    T.idst[i] = a.in_dst[mo + i];
    T.oq[i] = a.out_q[mo + i];
    T.odst[i] = a.out_dst[mo + i];
  }
  for (int i = lane; i <= a.P; i += 64) {
    T.iptr[i] = a.in_ptr[po + i];
    T.optr[i] = a.out_ptr[po + i];
  }
  for (int i = lane; i < a.P; i += 64) T.deg[i] = a.deg[(long)t * a.P + i];
  cl_wave_sync();
}

}  // namespace gsc
