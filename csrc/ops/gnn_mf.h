// Shared MFMA helpers of the fused GATv2 kernels (gnn_mf.hip: one wave per <= 32-node graph;
// gnn_mt.hip: one 32-node tile per wave, one graph per workgroup): bf16 fragment types, the
// v_mfma_f32_32x32x16_bf16 wrapper, accumulator row mapping, order-preserving float keys for the LDS
// max atomics, weight-fragment staging, the node linears and accumulator packing.
#pragma once
#include "gnn_args.h"

namespace gsc {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kMfRS = 40;                       // bf16 row stride of [row][k < 32] images
constexpr int kMfVec = 128;                     // fp32 per block in LDS: bl[32], br[32], att[32], bias[32]
constexpr int kMfFlush = 2 * 32 * 32 + kMfVec;  // fp32 per block in the end-of-kernel gradient image
constexpr int kMfFragSet = 4 * 64 * 4;         // floats of one fragment set [Wl0 Wl1 Wr0 Wr1][lane] x 16 B
constexpr int kMfKeyNegInf = (int)0x807FFFFF;   // mf_key(-inf)

__device__ __forceinline__ f32x16 mf_mma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// row of accumulator register i in lane half hh (32x32 C/D layout); the column is lane & 31
__device__ __forceinline__ int mf_row(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }
// float -> int key with the same order (ds_max_i32 implements a float max)
__device__ __forceinline__ int mf_key(float f) {
  const int k = __float_as_int(f);
  return k >= 0 ? k : k ^ 0x7fffffff;
}
__device__ __forceinline__ float mf_unkey(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }
// lane id through an opaque asm: lane-derived LDS addresses are recomputed where they are used instead
// of being hoisted out of the graph / layer loops, where they exceed the register budget and spill
__device__ __forceinline__ int mf_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// 8 weights as one bf16 fragment: W is [H][Fi] fp32 (module layout).  !trans: W[row][col0 + j]
// (B operand of X = h W^T); trans: W[col0 + j][row] (B operand of dh = dX W).
__device__ __forceinline__ bf16x8 mf_wfrag(const float* W, int H, int Fi, int row, int col0, bool trans) {
  // clamped unconditional loads, masked after all are issued (a guarded load per element compiled to a
  // branch around each load and one L2 round trip per element: ~32 serial trips per workgroup start)
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = trans ? col0 + j : row, k = trans ? row : col0 + j;
    v[j] = W[(c < H && k < Fi) ? c * Fi + k : 0];
  }
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = trans ? col0 + j : row, k = trans ? row : col0 + j;
    f[j] = (__bf16)((c < H && k < Fi) ? v[j] : 0.f);
  }
  return f;
}

struct MfW {
  bf16x8 l[2], r[2];
};

__device__ __forceinline__ void mf_load_w(MfW& w, const ClArgs& a, const float* params, int b, bool trans, int lane) {
  const int Fi = b == 0 ? a.Fin : a.H;
  const float* src = params + cl_block_offset(b, a.Fin, a.H);
  const float* Wl = src;
  const float* Wr = src + a.H * Fi + a.H;
  const int r = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    w.l[s] = mf_wfrag(Wl, a.H, Fi, r, 16 * s + 8 * hh, trans);
    w.r[s] = mf_wfrag(Wr, a.H, Fi, r, 16 * s + 8 * hh, trans);
  }
}

__device__ __forceinline__ void mf_stage_vec(const ClArgs& a, float* V, const float* params = nullptr) {
  if (!params) params = a.params;
  for (int i = threadIdx.x; i < a.n_blocks * kMfVec; i += blockDim.x) {
    const int b = i / kMfVec, j = i - b * kMfVec, which = j >> 5, c = j & 31;
    const int Fi = b == 0 ? a.Fin : a.H;
    const float* src = params + cl_block_offset(b, a.Fin, a.H);
    const int off = which == 0 ? a.H * Fi : (which == 1 ? 2 * a.H * Fi + a.H : 2 * a.H * Fi + a.H * which);
    const float x = src[off + (c < a.H ? c : 0)];
    V[i] = c < a.H ? x : 0.f;
  }
}

// Weight fragments staged once per workgroup, lane-linear (conflict-free ds_read_b128): set 0 =
// encoder, 1 = process block, 2 = process block transposed (backward's dh).  Read back per layer
// (mf_frags) instead of living in VGPRs for the whole kernel.
__device__ __forceinline__ void mf_stage_frags(const ClArgs& a, bf16x8* img, int nsets, const float* params = nullptr) {
  if (!params) params = a.params;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  for (int f = wave; f < nsets; f += waves) {
    MfW w;
    mf_load_w(w, a, params, f == 0 ? 0 : 1, f == 2, lane);
    img[(f * 4 + 0) * 64 + lane] = w.l[0];
    img[(f * 4 + 1) * 64 + lane] = w.l[1];
    img[(f * 4 + 2) * 64 + lane] = w.r[0];
    img[(f * 4 + 3) * 64 + lane] = w.r[1];
  }
}

__device__ __forceinline__ MfW mf_frags(const bf16x8* img, int b, int lane) {
  asm volatile("" ::: "memory");  // re-read per layer: keeps LICM from pinning 32 VGPRs for the whole loop
  MfW w;
  w.l[0] = img[(b * 4 + 0) * 64 + lane];
  w.l[1] = img[(b * 4 + 1) * 64 + lane];
  w.r[0] = img[(b * 4 + 2) * 64 + lane];
  w.r[1] = img[(b * 4 + 3) * 64 + lane];
  return w;
}

// Input rows -> bf16 image rows [rows][kMfRS] (and, SAVE_T, the transposed [k][node] image with row stride TS
// for k < trows): the images are cleared, then the nv valid rows -- nv * Fin contiguous floats -- are loaded
// four per lane at a time at clamped addresses (all in flight together) and scattered in.  (A
// per-element `v < n && k < Fin ? x[..] : 0` loop compiled to a branch around each load and waited for it:
// one HBM round trip per loop trip.)
template <bool SAVE_T>
__device__ __forceinline__ void mf_stage_input(const float* __restrict__ xg, int nv, int Fin, int rows, __bf16* hR,
                                               __bf16* hT, int TS, int trows, int lane) {
  const int nx = nv > 0 ? nv * Fin : 0;
  for (int i = lane; i < rows * 32; i += 64) {
    const int v = i >> 5, k = i & 31;
    hR[v * kMfRS + k] = (__bf16)0.f;
    if (SAVE_T && k < trows) hT[k * TS + v] = (__bf16)0.f;
  }
  for (int b0 = 0; b0 < nx; b0 += 256) {  // GSC shapes: one trip (11 x 3 or 32 x 3 floats)
    float xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = b0 + lane + 64 * u;
      xv[u] = xg[idx < nx ? idx : 0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = b0 + lane + 64 * u;
      if (idx < nx) {
        const int v = idx / Fin, k = idx - v * Fin;
        const __bf16 b = (__bf16)xv[u];
        hR[v * kMfRS + k] = b;
        if (SAVE_T) hT[k * TS + v] = b;
      }
    }
  }
}

__host__ __device__ __forceinline__ int mf_vec_floats(int n_blocks) { return n_blocks * kMfVec; }
// fp32 [node][channel] row stride (x_l, x_r, dy images): HPF + 4 floats = 16 B x odd, so the per-message
// row gathers (ds_read_b128 / b64 at different nodes) of up to 16 distinct rows hit distinct banks
__host__ __device__ constexpr int mf_xs(int HPF) { return HPF + 4; }

// X_l, X_r = h W^T + b: D[v][c] with lane column c and node rows in the 16 accumulators.
template <bool K2>
__device__ __forceinline__ void mf_linear(const MfW& w, const float* vec, const __bf16* h, int NV, int lane,
                                          f32x16& al, f32x16& ar) {
  const int r = lane & 31, hh = lane >> 5;
  const __bf16* hrow = h + (r < NV ? r : 0) * kMfRS + 8 * hh;
  const float blc = vec[r], brc = vec[32 + r];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    al[i] = blc;
    ar[i] = brc;
  }
  const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(hrow);
  al = mf_mma(a0, w.l[0], al);
  ar = mf_mma(a0, w.r[0], ar);
  if (K2) {
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(hrow + 16);
    al = mf_mma(a1, w.l[1], al);
    ar = mf_mma(a1, w.r[1], ar);
  }
}

// fp32 [node][HPF] image of an accumulator tile (rows < n) for the per-message VALU phases
template <int HPF>
__device__ __forceinline__ void mf_store_rows(const f32x16& acc, int n, float* img, int lane) {
  // one base address + compile-time row offsets (immediate ds_write offsets, no per-row registers)
  const int r = lane & 31, hh = lane >> 5;
  float* base = img + 4 * hh * mf_xs(HPF) + r;
  const int nn = n - 4 * hh;
  if (r < HPF) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ro = (i & 3) + 8 * (i >> 2);
      if (ro < nn) base[ro * mf_xs(HPF)] = acc[i];
    }
  }
}

__device__ __forceinline__ void mf_zero(f32x16& t) {
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0.f;
}
// sum of this lane's rows < n (lane column c; the two halves hold different rows)
__device__ __forceinline__ float mf_colsum(const f32x16& t, int nn) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((i & 3) + 8 * (i >> 2) < nn) s += t[i];
  return s;
}
// accumulator registers 8s..8s+7 as a bf16 fragment (rows 16s + 8(j>>2) + 4hh + (j&3))
__device__ __forceinline__ bf16x8 mf_pack(const f32x16& t, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)t[8 * s + j];
  return f;
}
// a [row][k] bf16 image read in the permuted k order that pairs with mf_pack: k = 16s + 4hh + (0..3)
// and 16s + 8 + 4hh + (0..3)
__device__ __forceinline__ bf16x8 mf_perm_frag(const __bf16* row, int s, int hh) {
  const bf16x4 e0 = *reinterpret_cast<const bf16x4*>(row + 16 * s + 4 * hh);
  const bf16x4 e1 = *reinterpret_cast<const bf16x4*>(row + 16 * s + 8 + 4 * hh);
  return __builtin_shufflevector(e0, e1, 0, 1, 2, 3, 4, 5, 6, 7);
}

struct MfVecGrad {
  float bl, br, bias;
};

}  // namespace gsc
