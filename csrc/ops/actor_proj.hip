// Fused actor output layer + critic action projection for large action spaces (the TD target's
// q'(s', clamp(mu'(s'), -1, 1)), reference simple_ddpg.py:205-207):
//
//   Z[m][j] = sum_n P[m][n] Wa[j][n],   P[m][n] = clamp((H[m] . W[n] + b[n]) * mask[topo[m]][n], lo, hi)
//
// H [M][K] is the actor's last hidden layer (bf16), W [A][K] its output weight, Wa [J][A] the
// critic's action block (J <= 64 units; rows zero-padded to a multiple of 8 columns, any A).  The [M, A] action matrix P is never written: per 64-column
// tile it lives in LDS between the two MFMA products (v_mfma_f32_32x32x16_bf16), so the HBM traffic
// is W and Wa once per XCD instead of writing and re-reading M x A bf16 (1.5 GB at M = 2048,
// A = 360,000: the materialised path took ~4 ms of the syn200 update).
//
// Workgroup = 8 waves over BM = 128 batch rows (4 x 2 waves of 32 x 32 for both products); each wave
// keeps the A fragments of its 32 H rows in registers for the whole walk (K <= 256: 16 fragments), so
// the first product reads only the W fragment from LDS (two 16-B LDS reads per MFMA with H in LDS put
// the kernel at the LDS read rate, 256 B/clk/CU, not the MFMA rate); it walks a contiguous range of
// action tiles with the W / Wa
// rows of the next PD tiles in flight in a register ring (the stream is latency-bound otherwise:
// one tile of MFMA work is ~0.5 us, an HBM round trip under load longer).  Grid = row blocks x
// S splits of the tiles; id = rb S + s with S a multiple of 8, so every row block of split s runs on
// XCD s mod 8 and they share the split's W / Wa stream in that XCD's L2.  Each split writes fp32
// partials [s][M][J]; splitk_reduce sums them in a fixed order (deterministic).
#include <hip/hip_bf16.h>
#include <pybind11/pybind11.h>

#include <cstdlib>

#include "../common.h"

namespace py = pybind11;

namespace gsc {
namespace aproj {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short s16x8;

constexpr int BM = 128;  // batch rows per workgroup
constexpr int BN = 64;   // action columns per tile
constexpr int NJ = 64;   // critic units (J <= NJ)
constexpr int NT = 512;  // threads
constexpr int LDP = BN + 4;  // Wa row stride (bf16): 34 words, so the 32 rows of a b64 fragment read land on 32 distinct
                             // bank pairs (BN + 8 = 36 words put rows r and r + 16 on the same banks)
constexpr int PD = 3;    // tiles in flight (register ring; 4 spilled once the H fragments moved to registers)

struct Args {
  const short* h;   // [M][ldh] bf16
  long ldh;
  const short* w;   // [A][ldw] bf16
  long ldw;
  const float* bias;  // [A]
  const float* mask;  // [T][ldm]
  long ldm;
  const int* topo;    // [M]
  const short* wa;    // [J][ldwa] bf16
  long ldwa;
  float* slabs;       // [S][M][J]
  int M, A, J, T, S, tiles, per_split;
  int A8;             // A rounded up to 8: Wa rows hold zero padding up to here (whole 16-byte chunks)
  float lo, hi;
};

__device__ __forceinline__ f32x16 mma(const s16x8& a, const s16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                 0);
}

__device__ __forceinline__ short f2bf(float f) { return (short)__bfloat16_as_ushort(__float2bfloat16(f)); }

// 16-byte chunk at (row r, column c0) with both clamped into the operand: every load is issued
// unconditionally (no branches around loads, so the compiler's vmcnt tracking keeps the prefetch
// ring in flight); the values that clamping duplicates are finite and multiplied by zero (mask
// columns beyond A or beyond the split, Z rows / columns beyond M / J are not stored).
__device__ __forceinline__ s16x8 load_chunk(const short* p, long ld, long r, long rows, long c0, long cols) {
  r = r < rows ? r : rows - 1;
  c0 = c0 + 8 <= cols ? c0 : cols - 8;
  return *reinterpret_cast<const s16x8*>(p + r * ld + c0);
}

constexpr int LDM = BN + 4;  // fp32 row stride of the staged mask rows (T rows: distinct banks)

// LDS bytes of the kernel: W double buffer [2][BN][K + 8] bf16, Wa double buffer [2][NJ][LDP] bf16, bias /
// mask double buffer [2][(1 + 4) LDM] fp32; the end-of-kernel partial exchange reuses the W buffers
template <int K>
constexpr size_t aproj_lds() {
  return sizeof(short) * (2 * BN * (K + 8) + 2 * NJ * LDP) + sizeof(float) * 2 * 5 * LDM;
}

// The first product is computed transposed, P^T[n][m] = W[n] . H[m] (A = W rows from LDS, B = the wave's
// resident H fragments): a lane then owns one batch row m (one topology: one mask row) and 16 action
// columns n in registers, and those registers ARE the A operand of the second product once the k order
// of each 16-wide step is permuted to the accumulator's row order (lane half hh holds n = 4 hh + 0..3 and
// 8 + 4 hh + 0..3; the Wa fragment is read in the same order with two 8-byte LDS reads).  P never goes
// through LDS: no P stores, no P barrier, and the epilogue is (acc + bias) * mask, clamp, bf16 per element.
// Each wave (wm, wn) accumulates Z[32 wm + .][0 .. 64) over its 32 columns of every tile; the two wn
// partials are added in a fixed order at the end (deterministic).
template <int K>
__global__ __launch_bounds__(NT) void actor_proj_kernel(Args a) {
  constexpr int LDK = K + 8;
  constexpr int KC = K / 8;                  // 16-byte chunks per row
  constexpr int WCH = BN * KC / NT;          // W tile chunks per thread
  static_assert(BN * KC % NT == 0 && BM * KC % NT == 0, "tile / thread mismatch");
  extern __shared__ __attribute__((aligned(16))) short ap_lds[];
  short* const s_w0 = ap_lds;                                       // [2][BN][LDK]
  short* const s_wa0 = s_w0 + 2 * BN * LDK;                         // [2][NJ][LDP]
  float* const s_v0 = reinterpret_cast<float*>(s_wa0 + 2 * NJ * LDP);  // [2][bias | mask t = 0..3][LDM]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int hh = lane >> 5, col = lane & 31;
  const int rb = blockIdx.x / a.S, split = blockIdx.x - rb * a.S;
  const long m0 = (long)rb * BM;
  const int t0 = split * a.per_split;
  const int t1 = min(a.tiles, t0 + a.per_split);

  // the lane's batch row (B column of the first product, A row of the second) and its topology
  const long mrow = m0 + 32 * wm + col;
  const int tp = a.topo[mrow < a.M ? mrow : a.M - 1] & 3;
  // resident B fragments of the wave's 32 H rows (column m = col, k = 16 s + 8 hh)
  s16x8 hf[K / 16];
#pragma unroll
  for (int s = 0; s < K / 16; ++s) hf[s] = load_chunk(a.h, a.ldh, mrow, a.M, 16 * s + 8 * hh, K);

  // register ring of PD tile stages: W / Wa chunks; threads < BN also the column's bias and masks
  s16x8 wreg[PD][WCH], areg[PD];
  float vst[PD][5];
  auto load_stage = [&](int d, int tt) {
    const long n0 = (long)(tt < a.tiles ? tt : a.tiles - 1) * BN;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int idx = tid + NT * i, r = idx / KC, c = idx - r * KC;
      wreg[d][i] = load_chunk(a.w, a.ldw, n0 + r, a.A, 8 * c, K);
    }
    const int r = tid >> 3, c = tid & 7;  // NJ x 8 chunks = 512
    areg[d] = load_chunk(a.wa, a.ldwa, r, a.J, n0 + 8 * c, a.A8);
    const long n = n0 + (tid & (BN - 1));
    const long nc = n < a.A ? n : a.A - 1;
    vst[d][0] = a.bias[nc];
#pragma unroll
    for (int t = 0; t < 4; ++t) vst[d][1 + t] = a.mask[(long)(t < a.T ? t : a.T - 1) * a.ldm + nc];
  };
  // a padding tile of the last group or a column beyond A gets mask 0 at the store (no wait at the load)
  auto store_stage = [&](int d, int buf, int tt) {
    short* sw = s_w0 + buf * BN * LDK;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int idx = tid + NT * i, r = idx / KC, c = idx - r * KC;
      *reinterpret_cast<s16x8*>(sw + r * LDK + 8 * c) = wreg[d][i];
    }
    const int r = tid >> 3, c = tid & 7;
    typedef __attribute__((ext_vector_type(4))) short s16x4w;
    short* wdst = s_wa0 + buf * NJ * LDP + r * LDP + 8 * c;  // 8-byte aligned rows (LDP = 68): two b64 stores
    *reinterpret_cast<s16x4w*>(wdst) = s16x4w{areg[d][0], areg[d][1], areg[d][2], areg[d][3]};
    *reinterpret_cast<s16x4w*>(wdst + 4) = s16x4w{areg[d][4], areg[d][5], areg[d][6], areg[d][7]};
    if (tid < BN) {
      const long n = (long)tt * BN + tid;
      const bool live = tt < t1 && n < a.A;
      float* v = s_v0 + buf * 5 * LDM;
      v[tid] = vst[d][0];
#pragma unroll
      for (int t = 0; t < 4; ++t) v[(1 + t) * LDM + tid] = live ? vst[d][1 + t] : 0.f;
    }
  };
  f32x16 acc2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[j][r] = 0.f;

#pragma unroll
  for (int d = 0; d < PD; ++d) load_stage(d, t0 + d);
  store_stage(0, 0, t0);
  __syncthreads();
  for (int tb = t0; tb < t1; tb += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int ti = tb + d;
      const int buf = (ti - t0) & 1;
      const short* sw = s_w0 + buf * BN * LDK;
      const short* swa = s_wa0 + buf * NJ * LDP;
      const float* sv = s_v0 + buf * 5 * LDM;
      // P^T tile: rows n = 32 wn + (i & 3) + 8 (i >> 2) + 4 hh, column m = col
      f32x16 acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[r] = 0.f;
#pragma unroll
      for (int s = 0; s < K / 16; ++s) {
        const s16x8 fw = *reinterpret_cast<const s16x8*>(sw + (32 * wn + col) * LDK + 16 * s + 8 * hh);
        acc1 = mma(fw, hf[s], acc1);
      }
      // epilogue in registers: (acc + bias[n]) * mask[tp][n], clamp, bf16 -> the second product's A operand
      s16x8 pa[2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nb = 32 * wn + 8 * q + 4 * hh;
        const float4 bv = *reinterpret_cast<const float4*>(sv + nb);
        const float4 mv = *reinterpret_cast<const float4*>(sv + (1 + tp) * LDM + nb);
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w}, mm[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = (acc1[4 * q + e] + bb[e]) * mm[e];
          v = fminf(fmaxf(v, a.lo), a.hi);
          pa[q >> 1][4 * (q & 1) + e] = f2bf(v);
        }
      }
      // Z[m][j] += sum_n P[m][n] Wa[j][n] over the wave's 32 columns (k order = the accumulator's row order)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          const short* wr = swa + (32 * jb + col) * LDP + 32 * wn + 16 * s2 + 4 * hh;
          typedef __attribute__((ext_vector_type(4))) short s16x4;
          const s16x4 lo4 = *reinterpret_cast<const s16x4*>(wr);
          const s16x4 hi4 = *reinterpret_cast<const s16x4*>(wr + 8);
          const s16x8 fb = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
          acc2[jb] = mma(pa[s2], fb, acc2[jb]);
        }
      }
      // tile ti + 1 into the other buffers (last read by tile ti - 1, before the previous barrier)
      store_stage((d + 1) % PD, buf ^ 1, ti + 1);
      load_stage(d, ti + PD);
      __syncthreads();
    }
  }
  // the two wn halves of every Z row block: wn = 1 parks its partial in LDS, wn = 0 adds it (fixed order)
  float* xch = reinterpret_cast<float*>(ap_lds) + wm * 32 * 64;  // [4][32 m][64 j] over the W buffers
  if (wn == 1) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 16; ++r) xch[((r & 3) + 8 * (r >> 2) + 4 * hh) * 64 + 32 * jb + col] = acc2[jb][r];
  }
  __syncthreads();
  if (wn == 0) {
    float* out = a.slabs + (long)split * a.M * a.J;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int j = 32 * jb + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mr = (r & 3) + 8 * (r >> 2) + 4 * hh;
        const long m = m0 + 32 * wm + mr;
        const float v = acc2[jb][r] + xch[mr * 64 + j];
        if (m < a.M && j < a.J) out[m * a.J + j] = v;
      }
    }
  }
}

void splitk_reduce_fwd(uintptr_t slabs, long slab, int splits, int M, int N, long lds_, uintptr_t out, long ldo,
                       float alpha, int accumulate, uintptr_t stream);

// Z (fp32 [M][J], row stride ldz) = sum over the action tiles; slabs >= S M J floats.
// Returns the split count used.
int actor_proj(uintptr_t h, long ldh, uintptr_t w, long ldw, uintptr_t bias, uintptr_t mask, long ldm, int T,
               uintptr_t topo, uintptr_t wa, long ldwa, int M, int K, int A, int J, float lo, float hi, uintptr_t slabs,
               long slab_floats, uintptr_t z, long ldz, uintptr_t stream) {
  GSC_CHECK(J >= 1 && J <= NJ, "actor_proj: at most 64 critic units");
  GSC_CHECK(T >= 1 && T <= 4, "actor_proj: at most 4 topologies");
  GSC_CHECK(K == 64 || K == 128 || K == 256, "actor_proj: actor width 64, 128 or 256");
  GSC_CHECK(A >= 8 && h % 16 == 0 && w % 16 == 0 && wa % 16 == 0 && ldh % 8 == 0 && ldw % 8 == 0 && ldwa % 8 == 0,
            "actor_proj: 16-byte aligned bf16 rows, A >= 8");
  // Wa's columns A .. round8(A) are read as part of the last 16-byte chunk: the caller keeps them zero
  // (rows padded to the stride), so ldwa >= round8(A)
  const int A8 = (A + 7) / 8 * 8;
  GSC_CHECK(ldwa >= A8, "actor_proj: Wa rows padded (zeros) to a multiple of 8 columns");
  const int rbs = (M + BM - 1) / BM;
  const int tiles = (A + BN - 1) / BN;
  // enough row blocks (large batches): one split, H read once and the whole W stream shared through
  // L2 -- unless the action space is long (>= 128 tiles: 50-node A = 22,500 is 352), where one split
  // left 200 workgroups walking every tile (1.2 ms at B = 25,600): 8 splits, one per XCD.  Small
  // batches: >= 256 workgroups with S a multiple of 8 (XCD grouping).
  int S = rbs >= 128 ? (tiles >= 128 ? 8 : 1) : ((256 + rbs - 1) / rbs + 7) / 8 * 8;
  if (rbs >= 128 && tiles >= 128) {
    // long action spaces at large batches: the multiple of 8 whose rbs x S workgroups (one per CU at a time) best
    // fill whole dispatch rounds, the smaller S within 1 % (config 5, rbs = 200: S = 8 left the 7th round a
    // quarter full, 7.26 ms; S = 32 fills 25 rounds, 6.62 ms; profiles/aproj_bench.txt)
    int dev = 0, cus = 256;
    GSC_HIP_CHECK(hipGetDevice(&dev));
    GSC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    double best = 0.0;
    for (int c = 8; c <= 64; c += 8) {
      if ((long)c * M * J > slab_floats || tiles / c < 64) break;  // >= 64 tiles per workgroup (H load amortised)
      const long wgs = (long)rbs * c, rounds = (wgs + cus - 1) / cus;
      const double eff = (double)wgs / (double)(rounds * cus);
      if (eff > best + 0.01) {
        best = eff;
        S = c;
      }
    }
  }
  static const int s_env = getenv("GSC_APROJ_SPLITS") ? atoi(getenv("GSC_APROJ_SPLITS")) : 0;  // tuning override
  if (s_env > 0) S = s_env;
  while (S > 1 && (long)S * M * J > slab_floats) S = S > 8 ? S - 8 : 1;
  GSC_CHECK((long)S * M * J <= slab_floats, "actor_proj: slabs too small");
  if (S > tiles) S = tiles;
  Args a{};
  a.h = ptr<const short>(h);
  a.ldh = ldh;
  a.w = ptr<const short>(w);
  a.ldw = ldw;
  a.bias = ptr<const float>(bias);
  a.mask = ptr<const float>(mask);
  a.ldm = ldm;
  a.topo = ptr<const int>(topo);
  a.wa = ptr<const short>(wa);
  a.ldwa = ldwa;
  a.slabs = ptr<float>(slabs);
  a.M = M;
  a.A = A;
  a.A8 = A8;
  a.J = J;
  a.T = T;
  a.S = S;
  a.tiles = tiles;
  a.per_split = (tiles + S - 1) / S;
  a.lo = lo;
  a.hi = hi;
  const hipStream_t s = stream_of(stream);
  const dim3 grid((unsigned)(rbs * S));
  static bool attr[3] = {false, false, false};  // > 64 KB of dynamic LDS: opted in once per width
  auto go = [&](auto kern, size_t lds, int slot) {
    if (!attr[slot]) {
      GSC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)lds));
      attr[slot] = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(NT), lds, s, a);
  };
  if (K == 256) go(actor_proj_kernel<256>, aproj_lds<256>(), 0);
  else if (K == 128) go(actor_proj_kernel<128>, aproj_lds<128>(), 1);
  else go(actor_proj_kernel<64>, aproj_lds<64>(), 2);
  check_launch();
  splitk_reduce_fwd(slabs, (long)M * J, S, M, J, J, z, ldz, 1.f, 0, stream);
  return S;
}

}  // namespace aproj

namespace mlp {
void splitk_reduce(uintptr_t slabs, long slab, int splits, int M, int N, long lds_, uintptr_t out, long ldo,
                   float alpha, int accumulate, uintptr_t stream);
}

namespace aproj {
void splitk_reduce_fwd(uintptr_t slabs, long slab, int splits, int M, int N, long lds_, uintptr_t out, long ldo,
                       float alpha, int accumulate, uintptr_t stream) {
  mlp::splitk_reduce(slabs, slab, splits, M, N, lds_, out, ldo, alpha, accumulate, stream);
}
}  // namespace aproj

void register_actor_proj(py::module_& m) {
  m.def("actor_proj", &aproj::actor_proj,
        "fused actor output layer (bias, per-topology mask, clamp) + critic action projection, no [M, A] matrix");
}

}  // namespace gsc
