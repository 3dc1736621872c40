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

// ---- critic products on the records: dense MFMA tiles expanded in LDS --------------------------------------------
// A row record expands to its P bf16 values (base below P, exceptions on top) with ~P/8 16-byte LDS stores and at
// most 11 two-byte ones, far cheaper per element than the 32x32x16 MFMA work it feeds (64 outputs per element), so
// both products run as bf16 MFMA GEMMs over one row block at a time: the replayed [B, A] block is never formed in
// memory (86 KB per transition read instead of 720 KB) and the MFMA time (B A c1 2 FLOP per pass) is the bound.
typedef __attribute__((ext_vector_type(8))) __bf16 sp_bf16x8;
typedef __attribute__((ext_vector_type(16))) float sp_f32x16;
typedef __attribute__((ext_vector_type(8))) short sp_s16x8;
typedef __attribute__((ext_vector_type(4))) short sp_s16x4;
typedef __attribute__((address_space(3))) sp_s16x4 sp_lds_s16x4;

constexpr int kSpC1 = 64;      // critic first-layer width (both products)
constexpr int kSpMaxFwdP = 240;  // forward LDS: 5 x [64][LD] bf16 images within 160 KB
constexpr int kSpBK = 64;      // samples per K step of the weight gradient

__device__ __forceinline__ sp_f32x16 sp_mma(const sp_s16x8& a, const sp_s16x8& b, const sp_f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(sp_bf16x8, a), __builtin_bit_cast(sp_bf16x8, b), c,
                                                 0, 0, 0);
}
// K-contiguous image row stride (elements): 4 x odd dwords, so the 16 rows of a ds_read_b128 lane group sit on
// 16 distinct bank quads
__host__ __device__ __forceinline__ int sp_ld_k(int Kp) { return (Kp / 8) % 2 ? Kp : Kp + 8; }
// M/N-contiguous image row stride for ds_read_b64_tr_b16 fragments: 2 LD mod 256 bytes in {64, 192}
__host__ __device__ __forceinline__ int sp_ld_tr(int C) { return (C / 32) % 2 ? C : C + 32; }

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

// Expand a record into chunks [ch0, ch1) (8 columns each) of an LDS row: base below P, zero from P on, then the
// record's exceptions inside the range (same lane, program order: they land after the base stores).  Row strides
// of 4 x odd dwords put the 8 lanes of a ds_write_b128 group on distinct bank quads.
__device__ __forceinline__ void sp_expand(short* row, const uint4& w0, const uint4& w1, const uint4& w2, int P,
                                          int ch0, int ch1) {
  const uint32_t head = w0.x, base = head & 0xffffu;
  const int cnt = (int)(head >> 16);
  const uint32_t bb = base | (base << 16);
  const int full = min(ch1, P >> 3);
  int c = ch0;
  for (; c < full; ++c) *reinterpret_cast<sp_u32x4*>(row + 8 * c) = sp_u32x4{bb, bb, bb, bb};
  for (; c < ch1; ++c) {  // the chunk holding column P (P % 8 != 0) and the zero padding after it
    sp_u32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = (8 * c + 2 * j < P ? base : 0u) | ((8 * c + 2 * j + 1 < P ? base : 0u) << 16);
    *reinterpret_cast<sp_u32x4*>(row + 8 * c) = v;
  }
  const uint32_t sl[kSpSlots] = {w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w};
  const int lo = 8 * ch0, hi = 8 * ch1;
#pragma unroll
  for (int k = 0; k < kSpSlots; ++k) {
    const int d = (int)(sl[k] & 0xffffu);
    if (k < cnt && d >= lo && d < hi) row[d] = (short)(sl[k] >> 16);
  }
}

// Records of the next D steps in registers (q[0] = this step's): a sampled record is a random HBM access, so its
// load is issued D - 1 steps before the expansion that reads it.
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
constexpr int kSpFwdDepth = 3;
constexpr int kSpWgradDepth = 4;

// Forward: part[s][b][:64] = sum_{r in split s} a[b, r P : r P + P] W_a[:, r P : r P + P]^T.
// 256 samples x one split of the row blocks per workgroup (4 waves x 64 samples, 64 x 64 outputs per wave).  Per
// row block: the W_a block [64][P] (aligned copy, zero past P) goes to a shared LDS image and every lane expands its
// sample's record into its wave's [64][P] image (no cross-wave dependence); the next block's W_a chunks and records
// are loaded into registers while the MFMAs run.  LDS: 5 x 64 x LD x 2 bytes (138 KB at P = 200).
// WVEC: P % 8 == 0 and 16-byte aligned W_a rows (16-byte loads of every chunk below P)
template <bool WVEC>
__global__ __launch_bounds__(256) void sparse_fwd_kernel(const uint32_t* __restrict__ ring, const int* __restrict__ rows,
                                                         int B, int R, int P, const __bf16* __restrict__ wa, long lda,
                                                         float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) short sp_lds[];
  const int Kp = (P + 15) & ~15, LD = sp_ld_k(Kp), CPR = Kp / 8, KS = Kp / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  short* Ws = sp_lds;                           // [64][LD]: W_a block (row = output o)
  short* As = sp_lds + (1 + wave) * 64 * LD;    // [64][LD]: this wave's 64 samples
  const int S = gridDim.y, sp = blockIdx.y;
  const int r_lo = (int)((long)R * sp / S), r_hi = (int)((long)R * (sp + 1) / S);
  const long b0 = (long)blockIdx.x * 256 + 64 * wave;
  const bool on = b0 + lane < B;
  const uint32_t* rec = ring + (long)(on ? rows[b0 + lane] : 0) * R * kSpWords;
  // W_a block: thread t loads row o = t / 4, chunks t % 4 + 4 i (CPR <= 30 chunks per row)
  constexpr int WPER = (kSpMaxFwdP / 8 + 3) / 4;
  const int wo = tid >> 2, wc = tid & 3;
  const __bf16* wrow = wa + (long)wo * lda;
  short* wdst = Ws + wo * LD + 8 * wc;
  sp_u32x4 wr[WPER];
  SpRecQueue<kSpFwdDepth> nq;
#pragma unroll
  for (int k = 0; k < kSpFwdDepth; ++k) {
    nq.clear(k);
    if (on && r_lo + k < r_hi) nq.fetch(k, rec + (long)(r_lo + k) * kSpWords);
  }
  auto load = [&](int r) {  // W_a block r
    const __bf16* src = wrow + (long)r * P + 8 * wc;
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int col = 8 * (wc + 4 * i);
      if (col >= 8 * CPR) break;
      if constexpr (WVEC) {
        wr[i] = col < P ? *reinterpret_cast<const sp_u32x4*>(src + 32 * i) : sp_u32x4{0, 0, 0, 0};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t x0 = col + 2 * j < P ? __builtin_bit_cast(uint16_t, src[32 * i + 2 * j]) : 0u;
          const uint32_t x1 = col + 2 * j + 1 < P ? __builtin_bit_cast(uint16_t, src[32 * i + 2 * j + 1]) : 0u;
          wr[i][j] = x0 | (x1 << 16);
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
  if (r_lo < r_hi) load(r_lo);
  const int r32 = lane & 31, h = lane >> 5;
  for (int r = r_lo; r < r_hi; ++r) {
    __syncthreads();  // the previous block's fragments are read
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      if (wc + 4 * i >= CPR) break;
      *reinterpret_cast<sp_u32x4*>(wdst + 32 * i) = wr[i];
    }
    sp_expand(As + lane * LD, nq.q[0][0], nq.q[0][1], nq.q[0][2], P, 0, CPR);
    if (r + 1 < r_hi) load(r + 1);
    nq.shift();
    if (on && r + kSpFwdDepth < r_hi) nq.fetch(kSpFwdDepth - 1, rec + (long)(r + kSpFwdDepth) * kSpWords);
    __syncthreads();
    for (int s = 0; s < KS; ++s) {
      sp_s16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const sp_s16x8*>(As + (32 * i + r32) * LD + 16 * s + 8 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const sp_s16x8*>(Ws + (32 * j + r32) * LD + 16 * s + 8 * h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = sp_mma(fa[i], fb[j], acc[i][j]);
    }
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
// (Np = P rounded up to 32: 2 x Np/32 tiles of 32 x 32, wave w owns column tiles w, w + 4 for both row tiles), K =
// the B samples in steps of 64: dh0 rows -> [64][96] and the 64 records expanded (4 threads per sample, a quarter
// of the row each) -> [64][LDB], both M/N-contiguous images read with ds_read_b64_tr_b16.  Every gradient element
// is written once (no atomics, deterministic); the next step's dh0 chunk and the records kSpWgradDepth - 1 steps
// ahead load during the MFMAs.
__global__ __launch_bounds__(256) void sparse_wgrad_kernel(const uint32_t* __restrict__ ring, const int* __restrict__ rows,
                                                           int B, int R, int P, const __bf16* __restrict__ dh0, long ldd,
                                                           float* __restrict__ gw, long ldg) {
  extern __shared__ __attribute__((aligned(16))) short sp_lds[];
  const int Np = (P + 31) & ~31, LDB = sp_ld_tr(Np), NT = Np / 32, CPQ = Np / 32;  // chunks per quarter row
  constexpr int LDA = 96;  // sp_ld_tr(64)
  short* Ai = sp_lds;                 // [64 samples][LDA]: dh0 (m = o)
  short* Bi = sp_lds + kSpBK * LDA;   // [64 samples][LDB]: expanded records (n = d)
  const int r = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int srow = tid >> 2, quarter = tid & 3;  // expansion: sample srow of the step, chunk quarter
  sp_u32x4 d0 = {0, 0, 0, 0}, d1 = d0;
  SpRecQueue<kSpWgradDepth> nq;
  auto fetch = [&](int k, int bs) {  // records of step bs into queue slot k
    const long b = bs + srow;
    if (b < B) nq.fetch(k, ring + ((long)rows[b] * R + r) * kSpWords);
    else nq.clear(k);
  };
  auto load = [&](int bs) {
    // dh0 chunk [64][64] bf16: 512 x 16 B, two per thread
    const int i0 = tid, i1 = tid + 256;
    const long ba = bs + (i0 >> 3), bb = bs + (i1 >> 3);
    d0 = ba < B ? *reinterpret_cast<const sp_u32x4*>(dh0 + ba * ldd + 8 * (i0 & 7)) : sp_u32x4{0, 0, 0, 0};
    d1 = bb < B ? *reinterpret_cast<const sp_u32x4*>(dh0 + bb * ldd + 8 * (i1 & 7)) : sp_u32x4{0, 0, 0, 0};
  };
#pragma unroll
  for (int k = 0; k < kSpWgradDepth; ++k) fetch(k, k * kSpBK);
  sp_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const bool t1 = wave + 4 < NT;  // second column tile of this wave
  const bool t0 = wave < NT;
  load(0);
  for (int bs = 0; bs < B; bs += kSpBK) {
    __syncthreads();
    *reinterpret_cast<sp_u32x4*>(Ai + (tid >> 3) * LDA + 8 * (tid & 7)) = d0;
    *reinterpret_cast<sp_u32x4*>(Ai + ((tid + 256) >> 3) * LDA + 8 * (tid & 7)) = d1;
    sp_expand(Bi + srow * LDB, nq.q[0][0], nq.q[0][1], nq.q[0][2], P, quarter * CPQ, quarter * CPQ + CPQ);
    if (bs + kSpBK < B) load(bs + kSpBK);
    nq.shift();
    fetch(kSpWgradDepth - 1, bs + kSpWgradDepth * kSpBK);
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
  const int col = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int d = 32 * (wave + 4 * j) + col;
    if (!(j == 0 ? t0 : t1) || d >= P) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int o = 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        gw[(long)o * ldg + (long)r * P + d] = acc[i][j][q];
      }
  }
}

static size_t sp_fwd_lds(int P) { return (size_t)5 * 64 * sp_ld_k((P + 15) & ~15) * 2; }
static size_t sp_wgrad_lds(int P) { return (size_t)kSpBK * (96 + sp_ld_tr((P + 31) & ~31)) * 2; }

static void sp_check(int R, int P, int c1 = 1) {
  GSC_CHECK(R > 0 && P > 0 && P <= 256, "sparse actions: 1..256 destinations per row");
  GSC_CHECK(c1 > 0 && c1 <= 256, "sparse actions: critic first layer width 1..256");
}

void register_sparse_act(py::module_& m) {
  m.attr("SPARSE_ACT_WORDS") = kSpWords;
  m.attr("SPARSE_ACT_SLOTS") = kSpSlots;
  m.def("sparse_compress", [](uintptr_t act, long ld, int E, int R, int P, uintptr_t ring, uintptr_t state,
                              long long cap, uintptr_t bad, uintptr_t stream) {
    sp_check(R, P);
    const long rows = (long)E * R;
    hipLaunchKernelGGL(sparse_compress_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream_of(stream),
                       ptr<const float>(act), ld, E, R, P, ptr<uint32_t>(ring), ptr<const long long>(state), cap,
                       ptr<int>(bad));
    check_launch();
  });
  // part: fp32 [splits, B, 64] partial sums (reduce with splitk_reduce); wa: the [64][lda] action block of W
  m.def("sparse_fwd", [](uintptr_t ring, uintptr_t rows, int B, int R, int P, uintptr_t wa, long lda, int c1,
                         uintptr_t part, int splits, uintptr_t stream) {
    sp_check(R, P, c1);
    GSC_CHECK(c1 == kSpC1, "sparse critic products: first layer width 64");
    GSC_CHECK(P <= kSpMaxFwdP, "sparse_fwd: at most 240 destinations per row");
    GSC_CHECK(splits >= 1 && splits <= R, "sparse_fwd: 1 <= splits <= R");
    GSC_CHECK(ring % 16 == 0, "sparse_fwd: 16-byte aligned record ring");
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
                         ptr<const int>(rows), B, R, P, ptr<const __bf16>(wa), lda, ptr<float>(part));
    else
      hipLaunchKernelGGL(sparse_fwd_kernel<false>, grid, dim3(256), lds, stream_of(stream), ptr<const uint32_t>(ring),
                         ptr<const int>(rows), B, R, P, ptr<const __bf16>(wa), lda, ptr<float>(part));
    check_launch();
  });
  m.def("sparse_wgrad", [](uintptr_t ring, uintptr_t rows, int B, int R, int P, uintptr_t dh0, long ldd, int c1,
                           uintptr_t gw, long ldg, uintptr_t stream) {
    sp_check(R, P, c1);
    GSC_CHECK(c1 == kSpC1, "sparse critic products: first layer width 64");
    GSC_CHECK(ring % 16 == 0 && dh0 % 16 == 0 && ldd % 8 == 0, "sparse_wgrad: 16-byte aligned ring and dh0 rows");
    const size_t lds = sp_wgrad_lds(P);
    hipLaunchKernelGGL(sparse_wgrad_kernel, dim3(R), dim3(256), lds, stream_of(stream), ptr<const uint32_t>(ring),
                       ptr<const int>(rows), B, R, P, ptr<const __bf16>(dh0), ldd, ptr<float>(gw), ldg);
    check_launch();
  });
}

}  // namespace gsc
