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
// Workgroup = 8 waves over BM = 128 batch rows (4 x 2 waves of 32 x 32 for both products); its H
// rows stay resident in LDS (K <= 256); it walks a contiguous range of action tiles with the W / Wa
// rows of the next PD tiles in flight in a register ring (the stream is latency-bound otherwise:
// one tile of MFMA work is ~0.5 us, an HBM round trip under load longer).  Grid = row blocks x
// S splits of the tiles; id = rb S + s with S a multiple of 8, so every row block of split s runs on
// XCD s mod 8 and they share the split's W / Wa stream in that XCD's L2.  Each split writes fp32
// partials [s][M][J]; splitk_reduce sums them in a fixed order (deterministic).
#include <hip/hip_bf16.h>
#include <pybind11/pybind11.h>

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
constexpr int LDP = BN + 8;
constexpr int PD = 4;    // tiles in flight (register ring)

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

template <int K>
__global__ __launch_bounds__(NT) void actor_proj_kernel(Args a) {
  constexpr int LDK = K + 8;
  constexpr int KC = K / 8;                  // 16-byte chunks per row
  constexpr int WCH = BN * KC / NT;          // W tile chunks per thread
  static_assert(BN * KC % NT == 0 && BM * KC % NT == 0, "tile / thread mismatch");
  __shared__ __attribute__((aligned(16))) short s_h[BM * LDK];
  __shared__ __attribute__((aligned(16))) short s_w[BN * LDK];
  __shared__ __attribute__((aligned(16))) short s_p[BM * LDP];
  __shared__ __attribute__((aligned(16))) short s_wa[2][NJ * LDP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int rb = blockIdx.x / a.S, split = blockIdx.x - rb * a.S;
  const long m0 = (long)rb * BM;
  const int t0 = split * a.per_split;
  const int t1 = min(a.tiles, t0 + a.per_split);

  // resident H rows
  for (int i = tid; i < BM * KC; i += NT) {
    const int r = i / KC, c = i - r * KC;
    *reinterpret_cast<s16x8*>(s_h + r * LDK + 8 * c) = load_chunk(a.h, a.ldh, m0 + r, a.M, 8 * c, K);
  }
  // topology of this lane's 16 accumulator rows (fixed for the workgroup)
  const int hh = lane >> 5, col = lane & 31;
  // packed 2 bits per row, formed before the tile loop (so no wait on these loads inside it)
  unsigned tpb = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * hh;
    tpb |= (unsigned)(a.topo[m < a.M ? m : a.M - 1] & 3) << (2 * r);
  }

  // register ring of PD tile stages (W / Wa rows, bias, mask column): tile ti + PD is requested right
  // after tile ti's P is built and stored to LDS PD - 1 tiles later, so the loads have PD - 1 tiles
  // of MFMA work to arrive
  s16x8 wreg[PD][WCH], areg[PD];
  float bst[PD], mst[PD][4];
  bool lst[PD];  // the stage's column is live (applied where the values are used: no wait at the load)
  // stage d <- tile tt (tt >= t1: a padding tile of the last group, its mask is zero)
  auto load_stage = [&](int d, int tt) {
    const long n0 = (long)(tt < a.tiles ? tt : a.tiles - 1) * BN;
    const long n = n0 + 32 * wn + col;
    const long nc = n < a.A ? n : a.A - 1;
    const bool live = tt < t1 && n < a.A;
    lst[d] = live;
    bst[d] = a.bias[nc];
#pragma unroll
    for (int t = 0; t < 4; ++t) mst[d][t] = a.mask[(long)(t < a.T ? t : a.T - 1) * a.ldm + nc];
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int idx = tid + NT * i, r = idx / KC, c = idx - r * KC;
      wreg[d][i] = load_chunk(a.w, a.ldw, n0 + r, a.A, 8 * c, K);
    }
    const int r = tid >> 3, c = tid & 7;  // NJ x 8 chunks = 512
    areg[d] = load_chunk(a.wa, a.ldwa, r, a.J, n0 + 8 * c, a.A8);
  };
  auto store_stage = [&](int d, int buf) {
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int idx = tid + NT * i, r = idx / KC, c = idx - r * KC;
      *reinterpret_cast<s16x8*>(s_w + r * LDK + 8 * c) = wreg[d][i];
    }
    const int r = tid >> 3, c = tid & 7;
    *reinterpret_cast<s16x8*>(&s_wa[buf][r * LDP + 8 * c]) = areg[d];
  };

  f32x16 acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;

#pragma unroll
  for (int d = 0; d < PD; ++d) load_stage(d, t0 + d);
  store_stage(0, 0);
  __syncthreads();
  // groups of PD tiles (the last group padded with zero-mask tiles: no branches around loads)
  for (int tb = t0; tb < t1; tb += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int ti = tb + d;
      {
        const int cur = (ti - t0) & 1;
        // P tile = epilogue(H W^T) for columns ti * 64 ..
        f32x16 acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc1[r] = 0.f;
#pragma unroll
        for (int s = 0; s < K / 16; ++s) {
          const s16x8 fa = *reinterpret_cast<const s16x8*>(s_h + (32 * wm + col) * LDK + 16 * s + 8 * hh);
          const s16x8 fb = *reinterpret_cast<const s16x8*>(s_w + (32 * wn + col) * LDK + 16 * s + 8 * hh);
          acc1 = mma(fa, fb, acc1);
        }
        const float bn = bst[d];
        const float mz0 = lst[d] ? mst[d][0] : 0.f, mz1 = lst[d] ? mst[d][1] : 0.f;
        const float mz2 = lst[d] ? mst[d][2] : 0.f, mz3 = lst[d] ? mst[d][3] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * hh;
          // two-level select on the topology bits (v_cndmask, no branches); topologies < T only
          const bool b0 = (tpb >> (2 * r)) & 1, b1 = (tpb >> (2 * r)) & 2;
          const float mlo = b0 ? mz1 : mz0, mhi = b0 ? mz3 : mz2;
          const float m = b1 ? mhi : mlo;
          float v = (acc1[r] + bn) * m;
          v = fminf(fmaxf(v, a.lo), a.hi);
          s_p[row * LDP + 32 * wn + col] = f2bf(v);
        }
        __syncthreads();  // P complete; every wave is done reading s_w
        store_stage((d + 1) % PD, cur ^ 1);
        load_stage(d, ti + PD);
        // Z += P Wa^T over the tile's 64 columns
#pragma unroll
        for (int s = 0; s < BN / 16; ++s) {
          const s16x8 fa = *reinterpret_cast<const s16x8*>(s_p + (32 * wm + col) * LDP + 16 * s + 8 * hh);
          const s16x8 fb = *reinterpret_cast<const s16x8*>(&s_wa[cur][(32 * wn + col) * LDP + 16 * s + 8 * hh]);
          acc2 = mma(fa, fb, acc2);
        }
        __syncthreads();  // done with P / Wa[cur]; the next tile's W / Wa are visible
      }
    }
  }
  // partial Z of this split
  float* out = a.slabs + (long)split * a.M * a.J;
  const int j = 32 * wn + col;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (m < a.M && j < a.J) out[m * a.J + j] = acc2[r];
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
  if (K == 256) hipLaunchKernelGGL(actor_proj_kernel<256>, grid, dim3(NT), 0, s, a);
  else if (K == 128) hipLaunchKernelGGL(actor_proj_kernel<128>, grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(actor_proj_kernel<64>, grid, dim3(NT), 0, s, a);
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
