// Sparse replayed actions for large action spaces (50- and 200-node topologies: A = N^2 C F).
//
// The replay buffer stores the *post-processed* action (reference simple_ddpg.py:291,300 store the output of
// post_process_actions, :374-395).  Post-processing is, per slice of n_pad destination weights, twice
// "zero entries < 0.1, renormalise to sum 1 (all-zero -> uniform 1/n_pad), add the rounding residual to the
// first entry that can absorb it".  The second pass's input sums to 1, so at most 10 entries survive its
// threshold; the residual may land on one more (an entry that was zero).  Every stored row is therefore
// either uniform (one value, the first entry possibly off by the residual) or has at most 11 non-zeros:
//
//   row record (12 x u32): word 0 = base value (bf16 bits) | exception count << 16
//                          words 1..11 = (destination index u16 | bf16 value << 16), ascending index
//
// and dense[d] = the exception's value where one is listed, else base -- exactly the bf16 row the dense ring
// held (compressed from the same fp32 -> bf16 rounding).  A syn200 transition: 1,800 rows x 48 B = 86 KB
// instead of 720 KB, so the ring can hold mem_limit transitions per env.
//
// The critic's two products over the replayed [B, A] block (h = a W_a^T and dW_a = dh0^T a) run as bf16 MFMA GEMMs
// one row block (P columns) at a time, with each sampled record expanded to its dense P values in LDS just before
// its fragments are read: the dense passes streamed 18.4 GB each at syn200, these read 2.2 GB of records.
#include <pybind11/pybind11.h>

#include <cstdlib>

#include <type_traits>

#include "../common.h"

namespace py = pybind11;

namespace gsc {

constexpr int kSpSlots = 11;  // exceptions per row
constexpr int kSpWords = 12;  // header + slots

__device__ __forceinline__ uint16_t bf16_bits(float x) {
  const __bf16 b = (__bf16)x;  // round to nearest even, as the dense ring's fp32 -> bf16 insert
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf16_val(uint32_t bits16) {
  return __builtin_bit_cast(float, (uint32_t)(bits16 & 0xffffu) << 16);
}

// One wave per (env, row): P <= 256 destinations, four per lane (index 64 q + lane).  Rows go to ring slot
// (pos + e) % cap (pos = the replay cursor before this insert's advance).  *bad counts rows with more than
// kSpSlots exceptions for both candidate bases (impossible for post-processed actions; checked by the caller).
__global__ __launch_bounds__(256) void sparse_compress_kernel(const float* __restrict__ act, long ld, int E, int R, int P,
                                                              uint32_t* __restrict__ ring,
                                                              const long long* __restrict__ state, long long cap,
                                                              int* __restrict__ bad) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)E * R) return;
  const int e = (int)(row / R), r = (int)(row - (long)e * R);
  const float* src = act + (long)e * ld + (long)r * P;
  uint16_t v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int d = 64 * q + lane;
    v[q] = d < P ? bf16_bits(src[d]) : (uint16_t)0;
  }
  // candidate bases: 0 (sparse rows) and the value at index 1 (uniform rows; index 0 may hold the residual)
  const uint16_t c1 = (uint16_t)__shfl((int)v[0], 1);
  int mis0 = 0, mis1 = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bool in = 64 * q + lane < P;
    mis0 += __popcll(__ballot(in && v[q] != 0));
    mis1 += __popcll(__ballot(in && v[q] != c1));
  }
  uint16_t base;
  int cnt;
  if (mis0 <= kSpSlots) { base = 0; cnt = mis0; }
  else if (mis1 <= kSpSlots) { base = c1; cnt = mis1; }
  else {  // not a post-processed row: keep the first kSpSlots non-base entries, flag it
    base = c1; cnt = kSpSlots;
    if (lane == 0) atomicAdd(bad, 1);
  }
  long long slot = state[0] + e;
  if (slot >= cap) slot -= cap;
  uint32_t* rec = ring + ((long)slot * R + r) * kSpWords;
  if (lane == 0) rec[0] = (uint32_t)base | ((uint32_t)cnt << 16);
  int k0 = 0;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bool ex = 64 * q + lane < P && v[q] != base;
    const unsigned long long m = __ballot(ex);
    const int k = k0 + __popcll(m & below);
    if (ex && k < cnt) rec[1 + k] = (uint32_t)(64 * q + lane) | ((uint32_t)v[q] << 16);
    k0 += __popcll(m);
  }
}

// The same records with one 16-byte load per lane (destinations 4 lane .. 4 lane + 3; P % 4 == 0, 16-byte aligned
// rows): the four-load lane-strided form above streamed the fp32 action block at ~1.9 TB/s.  Exceptions are listed in
// ascending destination order as there: lane-major, then the lane's four.
__global__ __launch_bounds__(256) void sparse_compress4_kernel(const float* __restrict__ act, long ld, int E, int R, int P,
                                                               uint32_t* __restrict__ ring,
                                                               const long long* __restrict__ state, long long cap,
                                                               int* __restrict__ bad) {
  const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (r >= R) return;
  const int e = blockIdx.y, lane = threadIdx.x & 63, d0 = 4 * lane;
  const float* src = act + (long)e * ld + (long)r * P;
  const bool on = d0 < P;
  const float4 f = *reinterpret_cast<const float4*>(src + (on ? d0 : 0));
  uint16_t v[4] = {bf16_bits(f.x), bf16_bits(f.y), bf16_bits(f.z), bf16_bits(f.w)};
  if (!on) v[0] = v[1] = v[2] = v[3] = 0;
  const uint16_t c1 = (uint16_t)__shfl((int)v[1], 0);  // the value at index 1 (lane 0's second)
  int mis0 = 0, mis1 = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mis0 += __popcll(__ballot(on && v[j] != 0));
    mis1 += __popcll(__ballot(on && v[j] != c1));
  }
  uint16_t base;
  int cnt;
  if (mis0 <= kSpSlots) { base = 0; cnt = mis0; }
  else if (mis1 <= kSpSlots) { base = c1; cnt = mis1; }
  else {
    base = c1; cnt = kSpSlots;
    if (lane == 0) atomicAdd(bad, 1);
  }
  long long slot = state[0] + e;
  if (slot >= cap) slot -= cap;
  uint32_t* rec = ring + ((long)slot * R + r) * kSpWords;
  if (lane == 0) rec[0] = (uint32_t)base | ((uint32_t)cnt << 16);
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int k = 0;  // exceptions of the lanes below this one
  bool ex[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ex[j] = on && v[j] != base;
    k += __popcll(__ballot(ex[j]) & below);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (ex[j]) {
      if (k < cnt) rec[1 + k] = (uint32_t)(d0 + j) | ((uint32_t)v[j] << 16);
      ++k;
    }
  }
}

// ---- critic products on the records: base column + sparse deltas in persistent LDS images ----------------------
// A row record is a rank-one part plus at most 11 point deltas: a[d] = base + delta[d], delta = v - base at the
// listed exceptions and zero elsewhere.  Both products run as bf16 MFMA GEMMs over one row block at a time on
// images that hold only the deltas plus ONE extra K column with the base value:
//
//   h[b] += sum_d a[b,d] W[:,d] = sum_d delta[b,d] W[:,d] + base_b * Wsum      (Wsum = sum_{d<P} W[:,d], per block)
//   dW[:,d] = sum_b dh0[b] a[b,d] = sum_b dh0[b] delta[b,d] + G,  G = sum_b dh0[b] base_b (the base column's output)
//
// The sample images stay zero between blocks: a lane writes its <= 11 deltas and its base column, the MFMAs read
// the image, and the same lane writes the deltas' positions back to zero -- ~24 two-byte LDS stores per sample
// and block instead of re-expanding the whole P-wide row (25 sixteen-byte stores at P = 200 plus the exceptions),
// which left the expansion and its barriers, not the MFMA, as the bound (round 5: sparse_fwd 3.0 ms, sparse_wgrad
// 3.6 ms of the syn200 step at 13-20 % of MFMA peak).  Wsum enters the forward as two bf16 columns (hi + lo part,
// each multiplied by base: ~2^-17 relative), computed per call by sparse_wsum_kernel.  delta = v - base is rounded
// to bf16 (exact for the sparse rows, base 0; one bf16 rounding of the residual on uniform rows).
typedef __attribute__((ext_vector_type(8))) __bf16 sp_bf16x8;
typedef __attribute__((ext_vector_type(16))) float sp_f32x16;
typedef __attribute__((ext_vector_type(8))) short sp_s16x8;
typedef __attribute__((ext_vector_type(4))) short sp_s16x4;
typedef __attribute__((address_space(3))) sp_s16x4 sp_lds_s16x4;

constexpr int kSpC1 = 64;        // critic first-layer width (both products)
constexpr int kSpMaxP = 238;     // forward LDS: 5 x [64][LD] bf16 images within 160 KB (K = P + 2 base columns)
constexpr int kSpBK = 64;        // samples per K step of the weight gradient

__device__ __forceinline__ sp_f32x16 sp_mma(const sp_s16x8& a, const sp_s16x8& b, const sp_f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(sp_bf16x8, a), __builtin_bit_cast(sp_bf16x8, b), c,
                                                 0, 0, 0);
}
// K-contiguous image row stride (elements): 4 x odd dwords, so the 16 rows of a ds_read_b128 lane group sit on
// 16 distinct bank quads
__host__ __device__ __forceinline__ int sp_ld_k(int Kp) { return (Kp / 8) % 2 ? Kp : Kp + 8; }
// M/N-contiguous image row stride for ds_read_b64_tr_b16 fragments: 2 LD mod 256 bytes in {64, 192}
__host__ __device__ __forceinline__ int sp_ld_tr(int C) { return (C / 32) % 2 ? C : C + 32; }
// forward K extent: P destinations + the two base columns, in whole 16-column MFMA steps
__host__ __device__ __forceinline__ int sp_kp_fwd(int P) { return (P + 2 + 15) & ~15; }
// weight-gradient N extent: P destinations + the base column, in whole 32-column tiles
__host__ __device__ __forceinline__ int sp_np_wgrad(int P) { return (P + 1 + 31) & ~31; }

// 32x32x16 fragment of a [k][c] (M/N-contiguous) image: lane = column (c0 + lane & 31), 8 k values (mlp.hip frag)
__device__ __forceinline__ sp_s16x8 sp_frag_tr(const short* img, int LD, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k = 16 * s + 8 * (g >> 1) + q;
  const short* a0 = img + k * LD + c0 + 16 * (g & 1) + 4 * p;
  const sp_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((sp_lds_s16x4*)(a0));
  const sp_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((sp_lds_s16x4*)(a0 + 4 * LD));
  return sp_s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

typedef __attribute__((ext_vector_type(4))) uint32_t sp_u32x4;  // 16-byte LDS stores (ds_write_b128)

// slot k of a record held as three uint4 (header word first)
__device__ __forceinline__ uint32_t sp_slot(const uint4& w0, const uint4& w1, const uint4& w2, int k) {
  const uint32_t sl[kSpSlots] = {w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w};
  return sl[k];
}
// bf16 bits of (v - base), v and base bf16 bits
__device__ __forceinline__ short sp_delta(uint32_t v, uint32_t base) {
  return (short)bf16_bits(bf16_val(v) - bf16_val(base));
}

// Records of the next D steps in registers (q[0] = this step's): a sampled record is a random HBM access, so its
// load is issued D - 1 steps before the step that reads it.
template <int D>
struct SpRecQueue {
  uint4 q[D][3];
  __device__ __forceinline__ void clear(int k) { q[k][0] = q[k][1] = q[k][2] = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ void fetch(int k, const uint32_t* rec) {
    const uint4* rp = reinterpret_cast<const uint4*>(rec);
    q[k][0] = rp[0]; q[k][1] = rp[1]; q[k][2] = rp[2];
  }
  __device__ __forceinline__ void shift() {
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
      q[k][0] = q[k + 1][0]; q[k][1] = q[k + 1][1]; q[k][2] = q[k + 1][2];
    }
  }
};
constexpr int kSpFwdW = 3;  // W_a blocks and records in flight (forward)

// Wsum of every row block: out[r][o] = bf16 hi | bf16 lo << 16 of sum_{d<P} W_a[o][r P + d] (fp32, fixed order).
// One wave per (r, o): four destinations per lane, DPP-free shuffle tree.
__global__ __launch_bounds__(256) void sparse_wsum_kernel(const __bf16* __restrict__ wa, long lda, int R, int P,
                                                          uint32_t* __restrict__ out) {
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= (long)R * kSpC1) return;
  const int r = (int)(w / kSpC1), o = (int)(w - (long)r * kSpC1);
  const __bf16* src = wa + (long)o * lda + (long)r * P;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int d = 64 * q + lane;
    if (d < P) s += (float)src[d];
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) {
    const uint32_t hi = bf16_bits(s);
    const uint32_t lo = bf16_bits(s - bf16_val(hi));
    out[(long)r * kSpC1 + o] = hi | (lo << 16);
  }
}

// Forward: part[s][b][:64] = sum_{r in split s} a[b, r P : r P + P] W_a[:, r P : r P + P]^T.
// 256 samples x one split of the row blocks per workgroup (4 waves x 64 samples, 64 x 64 outputs per wave).  Per
// row block: the W_a block [64][P] plus its two Wsum columns goes to a shared LDS image; every lane writes its
// sample's deltas and base columns into its wave's persistent [64][Kp] image and clears the deltas after the
// MFMAs (the wave's own LDS operations run in order); the next block's W_a chunks and records load into registers
// while the MFMAs run.  LDS: 5 x 64 x LD x 2 bytes (138 KB at P = 200).
// WVEC: P % 8 == 0 and 16-byte aligned W_a rows (16-byte loads of every chunk below P)
template <bool WVEC>
__global__ __launch_bounds__(256) void sparse_fwd_kernel(const uint32_t* __restrict__ ring, const int* __restrict__ rows,
                                                         int B, int R, int P, const __bf16* __restrict__ wa, long lda,
                                                         const uint32_t* __restrict__ wsum, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) short sp_lds[];
  const int Kp = sp_kp_fwd(P), LD = sp_ld_k(Kp), CPR = Kp / 8, KS = Kp / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  short* Ws = sp_lds;                           // [64][LD]: W_a block (row = output o)
  short* As = sp_lds + (1 + wave) * 64 * LD;    // [64][LD]: this wave's 64 samples
  short* myrow = As + lane * LD;
  const int S = gridDim.y, sp = blockIdx.y;
  const int r_lo = (int)((long)R * sp / S), r_hi = (int)((long)R * (sp + 1) / S);
  const long b0 = (long)blockIdx.x * 256 + 64 * wave;
  const bool on = b0 + lane < B;
  const uint32_t* rec = ring + (long)(on ? rows[b0 + lane] : 0) * R * kSpWords;
  for (int c = 0; c < CPR; ++c) *reinterpret_cast<sp_u32x4*>(myrow + 8 * c) = sp_u32x4{0, 0, 0, 0};
  // W_a block: thread t loads row o = t / 4, chunks t % 4 + 4 i (CPR <= 30 chunks per row)
  constexpr int WPER = ((kSpMaxP + 2 + 15) / 16 * 2 + 3) / 4;
  const int wo = tid >> 2, wc = tid & 3;
  const __bf16* wrow = wa + (long)wo * lda;
  short* wdst = Ws + wo * LD + 8 * wc;
  // W_a blocks of the next kSpFwdW row blocks in a register ring (set r mod kSpFwdW): a block is shared by the
  // workgroups of one split, whose first read of it misses in L2, and one MFMA phase (~0.7 us) did not cover
  // that latency (round 6: 17 % MFMA-busy with a one-block lead)
  sp_u32x4 wr[kSpFwdW][WPER];
  uint32_t ws[kSpFwdW];  // this thread's row o: Wsum hi | lo of the block in wr (stored by the wc == 0 thread)
  SpRecQueue<kSpFwdW> nq;  // this lane's records of the same blocks (set r mod kSpFwdW; no register shifting)
#pragma unroll
  for (int k = 0; k < kSpFwdW; ++k) {
    nq.clear(k);
    if (on && r_lo + k < r_hi) nq.fetch(k, rec + (long)(r_lo + k) * kSpWords);
  }
  auto load = [&](auto set, int r) {  // W_a block r (zero beyond P) into ring set `set`
    constexpr int SET = decltype(set)::value;
    const __bf16* src = wrow + (long)r * P + 8 * wc;
    ws[SET] = wsum[(long)r * kSpC1 + wo];
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int col = 8 * (wc + 4 * i);
      if (col >= 8 * CPR) break;
      if constexpr (WVEC) {
        wr[SET][i] = col < P ? *reinterpret_cast<const sp_u32x4*>(src + 32 * i) : sp_u32x4{0, 0, 0, 0};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t x0 = col + 2 * j < P ? __builtin_bit_cast(uint16_t, src[32 * i + 2 * j]) : 0u;
          const uint32_t x1 = col + 2 * j + 1 < P ? __builtin_bit_cast(uint16_t, src[32 * i + 2 * j + 1]) : 0u;
          wr[SET][i][j] = x0 | (x1 << 16);
        }
      }
    }
  };
  sp_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  static_assert(kSpFwdW == 3, "ring prologue / loop below are written for three sets");
  if (r_lo < r_hi) load(std::integral_constant<int, 0>{}, r_lo);
  if (r_lo + 1 < r_hi) load(std::integral_constant<int, 1>{}, r_lo + 1);
  if (r_lo + 2 < r_hi) load(std::integral_constant<int, 2>{}, r_lo + 2);
  const int r32 = lane & 31, h = lane >> 5;
  auto block = [&](auto set, int r) {
    constexpr int SET = decltype(set)::value;
    __syncthreads();  // the previous block's W_a fragments are read
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      if (wc + 4 * i >= CPR) break;
      *reinterpret_cast<sp_u32x4*>(wdst + 32 * i) = wr[SET][i];
    }
    if (wc == 0) {  // the two Wsum columns (after the chunk stores of this row: same wave, in order)
      Ws[wo * LD + P] = (short)(ws[SET] & 0xffffu);
      Ws[wo * LD + P + 1] = (short)(ws[SET] >> 16);
    }
    const uint4 w0 = nq.q[SET][0], w1 = nq.q[SET][1], w2 = nq.q[SET][2];
    const uint32_t base = w0.x & 0xffffu;
    const int cnt = (int)(w0.x >> 16);
#pragma unroll
    for (int k = 0; k < kSpSlots; ++k) {
      const uint32_t e = sp_slot(w0, w1, w2, k);
      if (k < cnt) myrow[e & 0xffffu] = sp_delta(e >> 16, base);
    }
    myrow[P] = (short)base;
    myrow[P + 1] = (short)base;
    if (r + kSpFwdW < r_hi) {
      load(set, r + kSpFwdW);
      if (on) nq.fetch(SET, rec + (long)(r + kSpFwdW) * kSpWords);
    }
    __syncthreads();
    {
      // software-pipelined K walk: step s + 1's fragments are read before step s's MFMAs issue (one wave per
      // SIMD: nothing else hides the LDS latency)
      const short* pa = As + r32 * LD + 8 * h;
      const short* pb = Ws + r32 * LD + 8 * h;
      sp_s16x8 fa0 = *reinterpret_cast<const sp_s16x8*>(pa), fa1 = *reinterpret_cast<const sp_s16x8*>(pa + 32 * LD);
      sp_s16x8 fb0 = *reinterpret_cast<const sp_s16x8*>(pb), fb1 = *reinterpret_cast<const sp_s16x8*>(pb + 32 * LD);
      for (int s = 0; s < KS; ++s) {
        const sp_s16x8 a0 = fa0, a1 = fa1, b0_ = fb0, b1 = fb1;
        if (s + 1 < KS) {
          const int o = 16 * (s + 1);
          fa0 = *reinterpret_cast<const sp_s16x8*>(pa + o);
          fa1 = *reinterpret_cast<const sp_s16x8*>(pa + 32 * LD + o);
          fb0 = *reinterpret_cast<const sp_s16x8*>(pb + o);
          fb1 = *reinterpret_cast<const sp_s16x8*>(pb + 32 * LD + o);
        }
        acc[0][0] = sp_mma(a0, b0_, acc[0][0]);
        acc[0][1] = sp_mma(a0, b1, acc[0][1]);
        acc[1][0] = sp_mma(a1, b0_, acc[1][0]);
        acc[1][1] = sp_mma(a1, b1, acc[1][1]);
      }
    }
    // clear the deltas (this wave's fragment reads of its image are issued above: in order)
#pragma unroll
    for (int k = 0; k < kSpSlots; ++k) {
      const uint32_t e = sp_slot(w0, w1, w2, k);
      if (k < cnt) myrow[e & 0xffffu] = 0;
    }
  };
  for (int r = r_lo; r < r_hi; r += kSpFwdW) {
    block(std::integral_constant<int, 0>{}, r);
    if (r + 1 < r_hi) block(std::integral_constant<int, 1>{}, r + 1);
    if (r + 2 < r_hi) block(std::integral_constant<int, 2>{}, r + 2);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const long b = b0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (b < B) {
        float* out = part + ((long)sp * B + b) * kSpC1 + r32;
        out[0] = acc[i][0][q];
        out[32] = acc[i][1][q];
      }
    }
}

// Gradient: dW_a[o, r P + d] = sum_b dh0[b, o] a[b, r P + d].  One workgroup per row block r: output [64][Np]
// (Np = P + 1 rounded up to 32: 2 x Np/32 tiles of 32 x 32, wave w owns column tiles w, w + 4 for both row tiles),
// K = the B samples in steps of 64: dh0 rows -> [64][96] and the 64 records' deltas + base column (column P) ->
// the persistent [64][LDB] image, both M/N-contiguous images read with ds_read_b64_tr_b16.  Four threads per
// sample: thread `quarter` loads only the record words it writes (the header and slots quarter, quarter + 4,
// quarter + 8: four dwords), kSpWgQ steps ahead -- a sampled record is a random HBM access (~2 us under load)
// and a step's MFMAs take ~0.2 us, so the queue must cover ~10 steps (it covered 3 at 12 dwords per slot:
// 46 % of wave cycles waiting).  The previous step's deltas are cleared after the barrier that ends its MFMAs.
// Row blocks are grouped by XCD (workgroup i runs on XCD i mod 8 and takes block (i mod 8) R8 + i / 8), so the
// blocks in flight on one XCD are consecutive and share the records' cache lines in that XCD's L2 (48-byte
// records, 128-byte lines).  The base column's output G[o] = sum_b dh0[b, o] base_b is added to every
// destination at the end.  Every gradient element is written once (no atomics, deterministic).
constexpr int kSpWgQ = 10;
__global__ __launch_bounds__(256) void sparse_wgrad_kernel(const uint32_t* __restrict__ ring, const int* __restrict__ rows,
                                                           int B, int R, int P, const __bf16* __restrict__ dh0, long ldd,
                                                           float* __restrict__ gw, long ldg) {
  extern __shared__ __attribute__((aligned(16))) short sp_lds[];
  const int R8 = (R + 7) / 8;
  const int r = (int)(blockIdx.x % 8) * R8 + (int)(blockIdx.x / 8);
  if (r >= R) return;
  const int Np = sp_np_wgrad(P), LDB = sp_ld_tr(Np), NT = Np / 32;
  constexpr int LDA = 96;  // sp_ld_tr(64)
  short* Ai = sp_lds;                 // [64 samples][LDA]: dh0 (m = o)
  short* Bi = sp_lds + kSpBK * LDA;   // [64 samples][LDB]: deltas + base column (n = d)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int srow = tid >> 2, quarter = tid & 3;  // sample srow of the step, slots k = quarter mod 4
  short* brow = Bi + srow * LDB;
  for (int c = quarter; c < Np / 8; c += 4) *reinterpret_cast<sp_u32x4*>(brow + 8 * c) = sp_u32x4{0, 0, 0, 0};
  sp_u32x4 d0 = {0, 0, 0, 0}, d1 = d0;
  // record words of the next kSpWgQ steps: [header, slot quarter, slot quarter + 4, slot quarter + 8]
  uint32_t q[kSpWgQ][4];
  auto fetch = [&](int k, int bs) {
    const long b = bs + srow;
    if (b < B) {
      const uint32_t* rec = ring + ((long)rows[b] * R + r) * kSpWords;
      q[k][0] = rec[0];
      q[k][1] = rec[1 + quarter];
      q[k][2] = rec[5 + quarter];
      q[k][3] = quarter < 3 ? rec[9 + quarter] : 0u;
    } else {
      q[k][0] = q[k][1] = q[k][2] = q[k][3] = 0u;
    }
  };
  auto load = [&](int bs) {
    // dh0 chunk [64][64] bf16: 512 x 16 B, two per thread
    const int i0 = tid, i1 = tid + 256;
    const long ba = bs + (i0 >> 3), bb = bs + (i1 >> 3);
    d0 = ba < B ? *reinterpret_cast<const sp_u32x4*>(dh0 + ba * ldd + 8 * (i0 & 7)) : sp_u32x4{0, 0, 0, 0};
    d1 = bb < B ? *reinterpret_cast<const sp_u32x4*>(dh0 + bb * ldd + 8 * (i1 & 7)) : sp_u32x4{0, 0, 0, 0};
  };
#pragma unroll
  for (int k = 0; k < kSpWgQ; ++k) fetch(k, k * kSpBK);
  sp_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[i][j][t] = 0.f;
  const bool t1 = wave + 4 < NT;  // second column tile of this wave
  const bool t0 = wave < NT;
  uint32_t prev[4] = {0u, 0u, 0u, 0u};  // the previous step's words (its deltas to clear)
  load(0);
  for (int bs = 0; bs < B; bs += kSpBK) {
    __syncthreads();  // the previous step's fragments are read
    *reinterpret_cast<sp_u32x4*>(Ai + (tid >> 3) * LDA + 8 * (tid & 7)) = d0;
    *reinterpret_cast<sp_u32x4*>(Ai + ((tid + 256) >> 3) * LDA + 8 * (tid & 7)) = d1;
    {
      const int pc = (int)(prev[0] >> 16);
#pragma unroll
      for (int m = 0; m < 3; ++m)
        if (quarter + 4 * m < pc) brow[prev[1 + m] & 0xffffu] = 0;
      const uint32_t base = q[0][0] & 0xffffu;
      const int cnt = (int)(q[0][0] >> 16);
#pragma unroll
      for (int m = 0; m < 3; ++m)
        if (quarter + 4 * m < cnt) brow[q[0][1 + m] & 0xffffu] = sp_delta(q[0][1 + m] >> 16, base);
      if (quarter == 0) brow[P] = (short)base;
#pragma unroll
      for (int m = 0; m < 4; ++m) prev[m] = q[0][m];
    }
    if (bs + kSpBK < B) load(bs + kSpBK);
#pragma unroll
    for (int k = 0; k + 1 < kSpWgQ; ++k)
#pragma unroll
      for (int m = 0; m < 4; ++m) q[k][m] = q[k + 1][m];
    fetch(kSpWgQ - 1, bs + kSpWgQ * kSpBK);
    __syncthreads();
    if (t0) {
#pragma unroll
      for (int s = 0; s < kSpBK / 16; ++s) {
        const sp_s16x8 fa0 = sp_frag_tr(Ai, LDA, 0, s, lane), fa1 = sp_frag_tr(Ai, LDA, 32, s, lane);
        const sp_s16x8 fb0 = sp_frag_tr(Bi, LDB, 32 * wave, s, lane);
        acc[0][0] = sp_mma(fa0, fb0, acc[0][0]);
        acc[1][0] = sp_mma(fa1, fb0, acc[1][0]);
        if (t1) {
          const sp_s16x8 fb1 = sp_frag_tr(Bi, LDB, 32 * (wave + 4), s, lane);
          acc[0][1] = sp_mma(fa0, fb1, acc[0][1]);
          acc[1][1] = sp_mma(fa1, fb1, acc[1][1]);
        }
      }
    }
  }
  // G[o] (the base column's output, column P: tile P / 32 of wave (P / 32) % 4, lanes P % 32 and P % 32 + 32)
  __syncthreads();
  float* G = reinterpret_cast<float*>(sp_lds);  // [64] (the dh0 image is no longer read)
  const int col = lane & 31, h = lane >> 5;
  {
    const int tp = P / 32, jp = tp / 4;
    if (wave == tp % 4 && col == P % 32) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 16; ++t) G[32 * i + (t & 3) + 8 * (t >> 2) + 4 * h] = jp ? acc[i][1][t] : acc[i][0][t];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int d = 32 * (wave + 4 * j) + col;
    if (!(j == 0 ? t0 : t1) || d >= P) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int o = 32 * i + (t & 3) + 8 * (t >> 2) + 4 * h;
        gw[(long)o * ldg + (long)r * P + d] = acc[i][j][t] + G[o];
      }
  }
}

static size_t sp_fwd_lds(int P) { return (size_t)5 * 64 * sp_ld_k(sp_kp_fwd(P)) * 2; }
static size_t sp_wgrad_lds(int P) { return (size_t)kSpBK * (96 + sp_ld_tr(sp_np_wgrad(P))) * 2; }

static void sp_check(int R, int P, int c1 = 1) {
  GSC_CHECK(R > 0 && P > 0 && P <= kSpMaxP, "sparse actions: 1..238 destinations per row");
  GSC_CHECK(c1 > 0 && c1 <= 256, "sparse actions: critic first layer width 1..256");
}

void register_sparse_act(py::module_& m) {
  m.attr("SPARSE_ACT_WORDS") = kSpWords;
  m.attr("SPARSE_ACT_SLOTS") = kSpSlots;
  m.def("sparse_compress", [](uintptr_t act, long ld, int E, int R, int P, uintptr_t ring, uintptr_t state,
                              long long cap, uintptr_t bad, uintptr_t stream) {
    sp_check(R, P);
    const long rows = (long)E * R;
    const char* ve = getenv("GSC_SP_COMPRESS4");  // 0: the lane-strided kernel (A/B)
    if (P % 4 == 0 && ld % 4 == 0 && act % 16 == 0 && E < 65536 && !(ve && ve[0] == '0'))
      hipLaunchKernelGGL(sparse_compress4_kernel, dim3((unsigned)((R + 3) / 4), (unsigned)E), dim3(256), 0,
                         stream_of(stream), ptr<const float>(act), ld, E, R, P, ptr<uint32_t>(ring),
                         ptr<const long long>(state), cap, ptr<int>(bad));
    else
      hipLaunchKernelGGL(sparse_compress_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream_of(stream),
                         ptr<const float>(act), ld, E, R, P, ptr<uint32_t>(ring), ptr<const long long>(state), cap,
                         ptr<int>(bad));
    check_launch();
  });
  // part: fp32 [splits, B, 64] partial sums (reduce with splitk_reduce); wa: the [64][lda] action block of W;
  // wsum: [R][64] uint32 scratch (the per-block column sums, written here)
  m.def("sparse_fwd", [](uintptr_t ring, uintptr_t rows, int B, int R, int P, uintptr_t wa, long lda, int c1,
                         uintptr_t wsum, uintptr_t part, int splits, uintptr_t stream) {
    sp_check(R, P, c1);
    GSC_CHECK(c1 == kSpC1, "sparse critic products: first layer width 64");
    GSC_CHECK(splits >= 1 && splits <= R, "sparse_fwd: 1 <= splits <= R");
    GSC_CHECK(ring % 16 == 0, "sparse_fwd: 16-byte aligned record ring");
    GSC_CHECK(wsum != 0 && wsum % 4 == 0, "sparse_fwd: a [R][64] uint32 scratch for the block sums");
    const long waves = (long)R * kSpC1;
    hipLaunchKernelGGL(sparse_wsum_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, stream_of(stream),
                       ptr<const __bf16>(wa), lda, R, P, ptr<uint32_t>(wsum));
    check_launch();
    const bool wvec = (wa % 16 == 0) && (lda % 8 == 0) && (P % 8 == 0);
    const size_t lds = sp_fwd_lds(P);
    static size_t attr[2] = {0, 0};
    const void* fn = wvec ? reinterpret_cast<const void*>(sparse_fwd_kernel<true>)
                          : reinterpret_cast<const void*>(sparse_fwd_kernel<false>);
    if (lds > 65536 && lds > attr[wvec]) {
      GSC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr[wvec] = lds;
    }
    const dim3 grid((B + 255) / 256, splits);
    if (wvec)
      hipLaunchKernelGGL(sparse_fwd_kernel<true>, grid, dim3(256), lds, stream_of(stream), ptr<const uint32_t>(ring),
                         ptr<const int>(rows), B, R, P, ptr<const __bf16>(wa), lda, ptr<const uint32_t>(wsum),
                         ptr<float>(part));
    else
      hipLaunchKernelGGL(sparse_fwd_kernel<false>, grid, dim3(256), lds, stream_of(stream), ptr<const uint32_t>(ring),
                         ptr<const int>(rows), B, R, P, ptr<const __bf16>(wa), lda, ptr<const uint32_t>(wsum),
                         ptr<float>(part));
    check_launch();
  });
  m.def("sparse_wgrad", [](uintptr_t ring, uintptr_t rows, int B, int R, int P, uintptr_t dh0, long ldd, int c1,
                           uintptr_t gw, long ldg, uintptr_t stream) {
    sp_check(R, P, c1);
    GSC_CHECK(c1 == kSpC1, "sparse critic products: first layer width 64");
    GSC_CHECK(ring % 16 == 0 && dh0 % 16 == 0 && ldd % 8 == 0, "sparse_wgrad: 16-byte aligned ring and dh0 rows");
    const size_t lds = sp_wgrad_lds(P);
    hipLaunchKernelGGL(sparse_wgrad_kernel, dim3(8 * ((R + 7) / 8)), dim3(256), lds, stream_of(stream), ptr<const uint32_t>(ring),
                       ptr<const int>(rows), B, R, P, ptr<const __bf16>(dh0), ldd, ptr<float>(gw), ldg);
    check_launch();
  });
}

}  // namespace gsc
