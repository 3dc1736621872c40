// Shared argument block of the fused MFMA GATv2 kernels (gnn_mf.hip, gnn_mt.hip; dispatched from gnn.hip).
#pragma once
#include "../common.h"

namespace gsc {

constexpr int kClMaxLayers = 16;
constexpr float kClSlope = 0.2f;

// Optional per-phase cycle counters (s_memtime); compiled out unless enabled at the call site.
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
  const void* s_dst;         // MFMA backward: bf16 [T, 32 * tiles, MP] one-hot target / source of each message
  const void* s_src;
  int MP;                    // messages padded to a multiple of 16
  void* blob;                // MFMA path: per-graph forward state saved for the backward (or null)
  const float* params2;      // forward only: a second parameter set on the same graphs (or null) ...
  float* emb2;               // ... and its embeddings [B, H] (target actor + target critic in one launch)
  int* work;                 // multi-tile backward: zeroed work-queue counter (graphs claimed by atomics), or null
  const int32_t* deg_order;  // [T, 2, P] nodes by in-degree / by out-degree, descending (large-graph kernels)
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
}  // namespace gsc
