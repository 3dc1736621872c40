// Hand-written bf16 MFMA GEMM engine for the DDPG actor/critic MLPs (gfx950, CDNA4).
//
//   C[M,N] = alpha * op(A)[M,K] . op(B)[K,N]   (fp32 accumulation on v_mfma_f32_32x32x16_bf16)
//
// Operand layouts (what the caller stores; the kernel never needs a transposed copy):
//   A_ROW  A stored [M][K] (activations)        A_COL  A stored [K][M] (dY^T of a weight gradient)
//   B_NK   B stored [N][K] (nn.Linear weight)   B_KN   B stored [K][N] (activations, W of dX = dY W)
// K-contiguous images are read as 16-byte fragments (ds_read_b128); M/N-contiguous images with the
// gfx950 hardware transpose read ds_read_b64_tr_b16 (two per 32x32x16 fragment), so every product of
// a DDPG update -- forward, input gradient, weight gradient -- is one kernel family.
//
// Block: 4 waves (256 threads), wave grid WM x WN, each wave owns (32 RM) x (32 RN) outputs; K is
// staged HBM/L2 -> registers -> LDS in BK-deep double-buffered tiles (the global loads of tile t+1
// are in flight while tile t is multiplied).  Edge tiles, fp32 operands (GNN embeddings, masks) and
// unaligned rows (the mask/action column blocks of the first-layer weights start at odd 16-byte
// offsets) take an element-wise staging path; interior tiles of aligned bf16 operands use 16-byte loads.
//
// Fused epilogue (in order): alpha, + bias[n], + rowtab[topo[m]][n] (per-topology mask fold of the
// first layer), + C32 (accumulate a previous K segment), * (gate[m][n] > 0) (ReLU derivative of a
// saved activation), ReLU, sigmoid (bounded actor output; its derivative s (1 - s) * colmask optionally
// written to dsig), * colmask[topo[m]][n] (actor output mask), * gmul[m][n] (a saved elementwise
// derivative: the sigmoid gate of the actor backward; may alias the bf16 output), clamp; bf16 and/or
// fp32 out.
// Split-K (gridDim.z > 1) writes raw fp32 slabs, summed by splitk_reduce in a fixed order
// (deterministic weight gradients, no atomics).
//
// Virtual B columns ("aug"): in B_KN operands, column N0 is a constant 1 and columns N0+1+t the
// one-hot of topo[k], so one weight-gradient GEMM dW = dY^T [X | 1 | onehot(topo)] also yields the
// bias gradient and the per-topology row sums that the folded mask block of W needs.
//
// Reference shapes: src/rlsp/agents/models.py:80-92 (critic MLP), 115-122 + 146-154 (actor MLP);
// the update math of simple_ddpg.py:204-234 is composed from these kernels in gsc_amd/ops/mlp.py.
#include <hip/hip_bf16.h>
#include <algorithm>
#include <pybind11/pybind11.h>

#include "../common.h"

namespace py = pybind11;

namespace gsc {
namespace mlp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

enum DType { DT_BF16 = 0, DT_F32 = 1 };

struct Operand {
  const void* p;
  long ld;       // elements between consecutive stored rows
  int dtype;     // DT_BF16 | DT_F32
  int vec;       // bf16, base 16-byte aligned, ld % 8 == 0: 16-byte loads of in-bounds chunks
  int vec32;     // fp32, base 16-byte aligned, ld % 4 == 0: two 16-byte loads per chunk (+ bf16 rounding)
  const int* rows;  // optional: stored row r is physical row rows[r] (replay-ring rows of a sampled batch read
                    // in place: the batch is never gathered into its own [B, A] copy)
};

struct Epilogue {
  float alpha;
  const float* bias;     // [N]
  const float* rowtab;   // [T][ld_rowtab] indexed by topo[m]
  long ld_rowtab;
  const int* topo;       // [M] (rowtab / colmask) -- for B aug columns: topo of the K rows
  const float* colmask;  // [T][ld_colmask]
  long ld_colmask;
  const __hip_bfloat16* gate;  // [M][ld_gate]: multiply by (gate > 0)
  long ld_gate;
  const float* rowscale;  // [M]: multiply row m
  const __hip_bfloat16* gmul;  // [M][ld_gmul]: multiply by gmul (read before c16 is written: may alias it)
  long ld_gmul;
  __hip_bfloat16* dsig;  // [M][ld_dsig]: sigmoid derivative s (1 - s) (* colmask) of the sigmoid epilogue
  long ld_dsig;
  int relu, clamp, accumulate, sigmoid;
  int single_topo;       // rowtab / colmask have one row (every topo[m] == 0): no per-row gathers
  int vec16;             // c16 base 16-byte aligned and ldc16 % 8 == 0: staged 16-byte row stores
  float lo, hi;
  float* c32;            // fp32 out (or split-K slabs)
  long ldc32;
  __hip_bfloat16* c16;   // bf16 out
  long ldc16;
};

struct GemmArgs {
  Operand a, b;
  int M, N, K;
  int kchunk;            // K per split (multiple of BK)
  long slab;             // split-K: elements between slabs of c32
  int aug_n0;            // >= 0: B_KN virtual columns start here (N0 = real columns), else -1
  int aug_t;             // number of one-hot topology columns after the ones column
  const int* aug_topo;   // topo of each K row (B_KN aug)
  Epilogue e;
};

__device__ __forceinline__ f32x16 mma(const s16x8& a, const s16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                 0);
}

__device__ __forceinline__ short f2bf(float f) {
  return (short)__bfloat16_as_ushort(__float2bfloat16(f));
}

__device__ __forceinline__ float bf2f(short s) { return __bfloat162float(__ushort_as_bfloat16((unsigned short)s)); }

__device__ __forceinline__ short load_elem(const Operand& o, long r, long c) {
  if (o.dtype == DT_F32) return f2bf(reinterpret_cast<const float*>(o.p)[r * o.ld + c]);
  return reinterpret_cast<const short*>(o.p)[r * o.ld + c];
}

// LDS row stride (elements) of an M/N-contiguous image: 2*LDT mod 256 bytes in {64, 192}, so the
// four rows of every ds_read_b64_tr_b16 block fall on disjoint bank ranges.
__host__ __device__ constexpr int tr_stride(int C) { return ((C / 32) % 2 == 1) ? C : C + 32; }

// K-contiguous images are [R][BK] with no row padding; the 16-byte chunk c of row r sits at chunk slot
// c ^ ((r / RP) & (BK / 8 - 1)), RP = 128 / BK rows per 64 banks.  Fragment reads (ds_read_b128, lane r =
// row r, all lanes the same chunk) then hit 16 distinct bank quads per lane group -- the 16 rows of a group
// are distinct mod 16 and (r mod RP, r / RP) spreads them over the 64 banks -- and the staging stores
// (ds_write_b128, 8 consecutive lanes = 32 contiguous dwords of one or two rows) cover the 32 store banks
// once.  A padded [R][BK + 8] image (the previous layout) serves the reads conflict-free but puts the
// second row of every store group on the first row's banks (2-way on every staging store).
template <int BK>
__device__ __forceinline__ int rowimg_off(int row, int ch) {
  constexpr int RP = 128 / BK, CPR = BK / 8;
  return row * BK + 8 * (ch ^ ((row / RP) & (CPR - 1)));
}

// Stage one operand tile into LDS.
//   ROWIMG: image [R][BK] (swizzled chunks, rowimg_off) of a K-contiguous operand (rows r0.., k0..)
//   !ROWIMG: image [BK][tr_stride(R)] of an M/N-contiguous operand (stored [k][c])
template <int R, int BK, bool ROWIMG>
struct Stager {
  static constexpr int CH = R * BK / 8;               // 16-byte chunks per tile
  static constexpr int PER = (CH + 255) / 256;        // chunks per thread
  s16x8 reg[PER];

  // rows_total/cols_total: extent of the stored matrix in (row, col) of the *stored* layout.  Each
  // 8-element chunk is loaded with vector loads when it is in bounds (per chunk, so the interior of
  // an edge tile stays vectorised); out-of-range elements are zero, aug columns are synthesised.
  __device__ __forceinline__ void load(const Operand& o, long srow0, long scol0, long rows_total, long cols_total,
                                       int tid, int aug_n0, int aug_t, const int* aug_topo) {
    constexpr int CPR = ROWIMG ? BK / 8 : R / 8;      // chunks per stored row inside the tile
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + 256 * i;
      if (CH % 256 != 0 && idx >= CH) break;
      const int row = idx / CPR, ch = idx % CPR;
      const long gr = srow0 + row, gc = scol0 + ch * 8;
      const bool inb = gr < rows_total && gc + 8 <= cols_total;
      const long pr = (o.rows && gr < rows_total) ? (long)o.rows[gr] : gr;  // physical row
      if (inb && o.vec) {
        reg[i] = *reinterpret_cast<const s16x8*>(reinterpret_cast<const short*>(o.p) + pr * o.ld + gc);
      } else if (inb && o.vec32) {
        const float4* src = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(o.p) + pr * o.ld + gc);
        const float4 x0 = src[0], x1 = src[1];
        reg[i] = s16x8{f2bf(x0.x), f2bf(x0.y), f2bf(x0.z), f2bf(x0.w), f2bf(x1.x), f2bf(x1.y), f2bf(x1.z),
                       f2bf(x1.w)};
      } else {
        s16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const long c = gc + j;
          short x = 0;
          if (gr < rows_total) {
            if (c < cols_total) x = load_elem(o, pr, c);
            else if (aug_n0 >= 0) {  // B_KN virtual columns: stored row = k (gr), column c
              const long t = c - aug_n0;
              if (t == 0) x = f2bf(1.f);
              else if (t >= 1 && t <= aug_t) x = f2bf(aug_topo[gr] == (int)(t - 1) ? 1.f : 0.f);
            }
          }
          v[j] = x;
        }
        reg[i] = v;
      }
    }
  }

  __device__ __forceinline__ void store(short* img, int tid) const {
    constexpr int CPR = ROWIMG ? BK / 8 : R / 8;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + 256 * i;
      if (CH % 256 != 0 && idx >= CH) break;
      const int row = idx / CPR, ch = idx % CPR;
      const int off = ROWIMG ? rowimg_off<BK>(row, ch) : row * tr_stride(R) + ch * 8;
      *reinterpret_cast<s16x8*>(img + off) = reg[i];
    }
  }
};

// Fragment of a 32x32x16 operand for k-step s, tile offset c0 (row of a ROWIMG image / column of a
// transposed image).  lane: r = lane & 31 (row of A / column of B), h = lane >> 5 (k half).
template <int R, int BK, bool ROWIMG>
__device__ __forceinline__ s16x8 frag(const short* img, int c0, int s, int lane) {
  if constexpr (ROWIMG) {
    const int r = lane & 31, h = lane >> 5;
    return *reinterpret_cast<const s16x8*>(img + rowimg_off<BK>(c0 + r, 2 * s + h));
  } else {
    constexpr int LD = tr_stride(R);
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = 16 * s + 8 * (g >> 1) + q;
    const int col = c0 + 16 * (g & 1) + 4 * p;
    const short* a0 = img + k * LD + col;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * LD));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <int RM, int RN, int WM, int WN, int BK, bool A_COL, bool B_KN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int BM = 32 * RM * WM, BN = 32 * RN * WN;
  constexpr int A_ELEMS = A_COL ? BK * tr_stride(BM) : BM * BK;
  constexpr int B_ELEMS = B_KN ? BK * tr_stride(BN) : BN * BK;
  // bf16 epilogue staging: per-wave [32 RM][32 RN] sub-tiles, unpadded (the 16-byte row-chunk reads of the
  // write-out then cover 64 distinct banks per lane group; a +8 pad put row 3 on row 0's banks)
  constexpr int LDT = 32 * RN;
  constexpr int OPS = 2 * (A_ELEMS + B_ELEMS), STG = 4 * (32 * RM) * LDT;
  __shared__ __attribute__((aligned(16))) short smem[OPS > STG ? OPS : STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long m0 = (long)blockIdx.x * BM, n0 = (long)blockIdx.y * BN;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  Stager<BM, BK, !A_COL> sa;
  Stager<BN, BK, !B_KN> sb;
  // stored-layout coordinates of the tiles: A_ROW (m, k), A_COL (k, m); B_NK (n, k), B_KN (k, n)
  auto load_tiles = [&](int kt) {
    const long k0 = kbeg + (long)kt * BK;
    if (A_COL) sa.load(g.a, k0, m0, kend, g.M, tid, -1, 0, nullptr);
    else sa.load(g.a, m0, k0, g.M, kend, tid, -1, 0, nullptr);
    if (B_KN) sb.load(g.b, k0, n0, kend, g.aug_n0 >= 0 ? g.aug_n0 : g.N, tid, g.aug_n0, g.aug_t, g.aug_topo);
    else sb.load(g.b, n0, k0, g.N, kend, tid, -1, 0, nullptr);
  };

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (ntiles > 0) {
    load_tiles(0);
    sa.store(smem, tid);
    sb.store(smem + A_ELEMS, tid);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int cur = kt & 1;
      const short* ia = smem + cur * (A_ELEMS + B_ELEMS);
      const short* ib = ia + A_ELEMS;
      if (kt + 1 < ntiles) load_tiles(kt + 1);
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        s16x8 fa[RM], fb[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) fa[i] = frag<BM, BK, !A_COL>(ia, wm * 32 * RM + 32 * i, s, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) fb[j] = frag<BN, BK, !B_KN>(ib, wn * 32 * RN + 32 * j, s, lane);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) acc[i][j] = mma(fa[i], fb[j], acc[i][j]);
      }
      if (kt + 1 < ntiles) {
        short* na = smem + (cur ^ 1) * (A_ELEMS + B_ELEMS);
        sa.store(na, tid);
        sb.store(na + A_ELEMS, tid);
      }
      __syncthreads();
    }
  }

  const Epilogue& e = g.e;
  const bool split = gridDim.z > 1;
  float* c32 = e.c32 ? e.c32 + (split ? (long)blockIdx.z * g.slab : 0) : nullptr;
  const int col_l = lane & 31, hh = lane >> 5;
  const bool per_row_topo = (e.rowtab || e.colmask) && !e.single_topo;
  // bf16 output through LDS (per-wave sub-tile, padded rows) when the output rows are 16-byte aligned
  const bool stage16 = !split && e.c16 && e.vec16;
  short* stile = smem + wave * (32 * RM) * LDT;
  if (stage16) __syncthreads();  // every wave is done reading the operand tiles
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    // topology of this lane's 16 rows, loaded once per row block (all gathers issued up front)
    int tp[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long m = m0 + wm * 32 * RM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
      tp[r] = (per_row_topo && m < g.M) ? e.topo[m] : 0;
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const long n = n0 + wn * 32 * RN + 32 * j + col_l;
      if (n >= g.N) continue;
      const float bn = (!split && e.bias) ? e.bias[n] : 0.f;
      // per-topology row tables: one value per column with a single topology, else gathered per row
      float rt[16], cm[16];
      if (!split && e.rowtab) {
        if (e.single_topo) {
          const float x = e.rowtab[n];
#pragma unroll
          for (int r = 0; r < 16; ++r) rt[r] = x;
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) rt[r] = e.rowtab[(long)tp[r] * e.ld_rowtab + n];
        }
      }
      if (!split && e.colmask) {
        if (e.single_topo) {
          const float x = e.colmask[n];
#pragma unroll
          for (int r = 0; r < 16; ++r) cm[r] = x;
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) cm[r] = e.colmask[(long)tp[r] * e.ld_colmask + n];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm * 32 * RM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m >= g.M) continue;
        float v = acc[i][j][r];
        if (split) {
          c32[m * e.ldc32 + n] = v;
          continue;
        }
        v = v * e.alpha + bn;
        if (e.rowtab) v += rt[r];
        if (e.accumulate) v += c32[m * e.ldc32 + n];
        if (e.gate && !(__bfloat162float(e.gate[m * e.ld_gate + n]) > 0.f)) v = 0.f;
        if (e.relu) v = v > 0.f ? v : 0.f;
        if (e.sigmoid) {
          v = 1.f / (1.f + __expf(-v));
          if (e.dsig) e.dsig[m * e.ld_dsig + n] = __float2bfloat16(e.colmask ? v * (1.f - v) * cm[r] : v * (1.f - v));
        }
        if (e.colmask) v *= cm[r];
        if (e.gmul) v *= __bfloat162float(e.gmul[m * e.ld_gmul + n]);
        if (e.rowscale) v *= e.rowscale[m];
        if (e.clamp) v = fminf(fmaxf(v, e.lo), e.hi);
        if (c32) c32[m * e.ldc32 + n] = v;
        if (e.c16) {
          if (stage16) stile[(32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh) * LDT + 32 * j + col_l] = f2bf(v);
          else e.c16[m * e.ldc16 + n] = __float2bfloat16(v);
        }
      }
    }
  }
  if (stage16) {
    // bf16 output staged through LDS: each lane stores 16 contiguous bytes of a row (full-line
    // writes instead of 2-byte column scatters)
    __builtin_amdgcn_wave_barrier();
    constexpr int CPR = 32 * RN / 8;  // 16-byte chunks per sub-tile row
    const long mb = m0 + wm * 32 * RM, nb = n0 + wn * 32 * RN;
    for (int idx = lane; idx < 32 * RM * CPR; idx += 64) {
      const int row = idx / CPR, ch = idx % CPR;
      const long m = mb + row, n = nb + 8 * ch;
      if (m >= g.M) continue;
      const short* src = stile + row * LDT + 8 * ch;
      if (n + 8 <= g.N) {
        *reinterpret_cast<s16x8*>(reinterpret_cast<short*>(e.c16) + m * e.ldc16 + n) =
            *reinterpret_cast<const s16x8*>(src);
      } else {
        for (int k = 0; k < 8 && n + k < g.N; ++k) reinterpret_cast<short*>(e.c16)[m * e.ldc16 + n + k] = src[k];
      }
    }
  }
}

// out[m][n] (row stride ldo) = alpha * sum_z slab[z][m][n] (+ out if accumulate).  A block takes 64
// consecutive outputs x 4 split phases (phase p sums splits p, p+4, ...), then adds the 4 phase sums
// in a fixed order: deterministic, and parallel over the splits when there are few outputs.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* slabs, long slab, int splits, int M, int N,
                                                            long lds_, float* out, long ldo, float alpha,
                                                            int accumulate) {
  __shared__ float red[4][64];
  const long total = (long)M * N;
  const int j = threadIdx.x & 63, ph = threadIdx.x >> 6;
  for (long base = (long)blockIdx.x * 64; base < total; base += (long)gridDim.x * 64) {
    const long i = base + j;
    float s = 0.f;
    long m = 0, n = 0;
    if (i < total) {
      m = i / N;
      n = i - m * N;
      const float* p = slabs + m * lds_ + n;
#pragma unroll 4
      for (int z = ph; z < splits; z += 4) s += p[(long)z * slab];
    }
    red[ph][j] = s;
    __syncthreads();
    if (ph == 0 && i < total) {
      float v = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
      v *= alpha;
      if (accumulate) v += out[m * ldo + n];
      out[m * ldo + n] = v;
    }
    __syncthreads();
  }
}

// out[t][n] (row stride ldo) = sum_a x[t][a] W[n][a]: the per-topology fold of a 0/1 mask block of a
// first-layer weight (x = masks [T][A], W = the mask columns) and small GEMVs (x = a bias vector).
// Grid (N, S): workgroup (n, z) reads row n of W once over its A-chunk for TT topologies at a time (W is
// the HBM stream; the x rows stay in L2), bf16 pairs when the row is 4-byte aligned.  S > 1 writes
// partials [S][T][N] for splitk_reduce (fixed order: deterministic).
// BITS: x is a 0/1 matrix given as packed bits (uint32 words, bit a % 32 of word a / 32, ldx words per
// row): the mask fold reads 1/32 of the fp32 mask bytes per W element (at A = 360,000 the fp32 masks,
// re-read from L2 by every row n, were the kernel's main traffic).  x_a w_a with x_a in {0, 1} is w_a
// or zero exactly, so the sums equal the fp32 path's (up to the sign of zero).
template <int TT, bool BITS>
__global__ __launch_bounds__(256) void rowdot_kernel(const float* x, long ldx, int T, const __hip_bfloat16* W,
                                                     long ldw, int N, int A, int achunk, int pair, float* out,
                                                     long ldo) {
  const uint32_t* xb = reinterpret_cast<const uint32_t*>(x);
  __shared__ float red[4][TT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x, z = blockIdx.y;
  const int a0 = z * achunk, a1 = min(A, a0 + achunk);
  const __hip_bfloat16* wr = W + (long)n * ldw;
  for (int t0 = 0; t0 < T; t0 += TT) {
    float s[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) s[t] = 0.f;
    if (pair) {
      for (int a = a0 + 2 * (int)threadIdx.x; a < a1; a += 512) {
        const __hip_bfloat162 w2 = *reinterpret_cast<const __hip_bfloat162*>(wr + a);
        const float w0 = __low2float(w2), w1 = a + 1 < a1 ? __high2float(w2) : 0.f;
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          if (t0 + t < T) {
            if constexpr (BITS) {
              const uint32_t wd = xb[(long)(t0 + t) * ldx + (a >> 5)] >> (a & 31);  // a even: a + 1 in the same word
              s[t] += ((wd & 1u) ? w0 : 0.f) + ((wd & 2u) ? w1 : 0.f);
            } else {
              const float2 xv = *reinterpret_cast<const float2*>(x + (long)(t0 + t) * ldx + a);
              s[t] += xv.x * w0 + xv.y * w1;
            }
          }
        }
      }
    } else {
      for (int a = a0 + (int)threadIdx.x; a < a1; a += 256) {
        const float w0 = __bfloat162float(wr[a]);
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          if (t0 + t >= T) continue;
          if constexpr (BITS) s[t] += ((xb[(long)(t0 + t) * ldx + (a >> 5)] >> (a & 31)) & 1u) ? w0 : 0.f;
          else s[t] += x[(long)(t0 + t) * ldx + a] * w0;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s[t] += __shfl_xor(s[t], off);
      if (lane == 0) red[wv][t] = s[t];
    }
    __syncthreads();
    if ((int)threadIdx.x < TT && t0 + (int)threadIdx.x < T) {
      const int t = threadIdx.x;
      const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
      if (gridDim.y == 1) out[(long)(t0 + t) * ldo + n] = v;
      else out[((long)z * T + t0 + t) * N + n] = v;  // partial slab z
    }
    __syncthreads();
  }
}

// dst[r][t C + c] = (topo[r] == t) ? src[r][c] : 0  (bf16): the per-topology block expansion of an
// activation / gradient, so a product with per-topology matrices becomes one GEMM over K = T C.
__global__ __launch_bounds__(256) void topo_expand_kernel(const __hip_bfloat16* src, long lds_, __hip_bfloat16* dst,
                                                          long ldd, int R, int C, int T, const int* topo) {
  const long total = (long)R * T * C;
  const int TC = T * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / TC), j = (int)(i - (long)r * TC);
    const int t = j / C, c = j - t * C;
    dst[(long)r * ldd + j] = topo[r] == t ? src[(long)r * lds_ + c] : __float2bfloat16(0.f);
  }
}

// ------------------------------------------------------------------------------------------------
// Critic output layer Linear(C, 1) with the DDPG losses fused (reference simple_ddpg.py:204-225):
//   mode 0 (TD target)   y = r + (1 - d) gamma q'                                    -> y[B]
//   mode 1 (critic loss) diff = q - y, dq = 2 diff / B, dh = dq w (h > 0)             -> dh, partials
//                        partials per wave: dw[c] = sum dq h[c], db = sum dq, sum diff^2, sum q
//   mode 2 (actor loss)  la = -mean q: dq = -1 / B, dh = dq w (h > 0)                 -> dh, sum q
// One wave per row at a time, lane = channel (CPL channels per lane), q by a wave butterfly.
// ------------------------------------------------------------------------------------------------
struct HeadArgs {
  const __hip_bfloat16* h;
  long ldh;
  int B, C, mode;
  const float* w;  // fp32 master weight [C]
  const float* b;  // [1]
  float gamma, inv_b;
  const float* r;
  const float* d;
  float* y;
  __hip_bfloat16* dh;
  long lddh;
  float* part;     // [blocks][C + 3]
};

template <int CPL>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  float w[CPL], dw[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = lane + 64 * k;
    w[k] = c < a.C ? a.w[c] : 0.f;
    dw[k] = 0.f;
  }
  const float bias = a.b[0];
  float db = 0.f, loss = 0.f, qsum = 0.f;
  for (int row = gw; row < a.B; row += nw) {
    float v[CPL], s = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      v[k] = c < a.C ? __bfloat162float(a.h[(long)row * a.ldh + c]) : 0.f;
      s += v[k] * w[k];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    const float q = s + bias;
    qsum += q;
    if (a.mode == 0) {
      if (lane == 0) a.y[row] = a.r[row] + (1.f - a.d[row]) * a.gamma * q;
      continue;
    }
    float dq;
    if (a.mode == 1) {
      const float diff = q - a.y[row];
      loss += diff * diff;
      dq = 2.f * diff * a.inv_b;
      db += dq;
    } else {
      dq = -a.inv_b;
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if (c < a.C) a.dh[(long)row * a.lddh + c] = __float2bfloat16(v[k] > 0.f ? dq * w[k] : 0.f);
      dw[k] += dq * v[k];
    }
  }
  if (a.part) {  // the block's 4 wave partials summed in a fixed order -> one row of the slab per block
    __shared__ float red[4][64 * CPL + 3];
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < CPL; ++k) red[wv][lane + 64 * k] = dw[k];
    if (lane == 0) {
      red[wv][64 * CPL] = db;
      red[wv][64 * CPL + 1] = loss;
      red[wv][64 * CPL + 2] = qsum;
    }
    __syncthreads();
    float* p = a.part + (long)blockIdx.x * (a.C + 3);
    for (int c = threadIdx.x; c < a.C + 3; c += blockDim.x) {
      const int src = c < a.C ? c : 64 * CPL + (c - a.C);
      p[c] = ((red[0][src] + red[1][src]) + red[2][src]) + red[3][src];
    }
  }
}

// Gradient of a first layer [N][ldw] from the augmented weight-gradient GEMM tmp [N][H + 1 + T]
// (columns: dense inputs, ones, topology one-hot):  gW[:, :H] = tmp[:, :H];  gb = tmp[:, H];
// gW[n][H + a] = sum_t tmp[n][H + 1 + t] mask[t][a]  (the folded mask block of the input).
__global__ __launch_bounds__(256) void first_layer_grad_kernel(const float* tmp, int N, int H, int T, int A,
                                                               const float* mask, long ldm, float* gW, long ldw,
                                                               float* gb) {
  const int W = H + A;
  const long total = (long)N * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / W), c = (int)(i - (long)n * W);
    const float* row = tmp + (long)n * (H + 1 + T);
    float v;
    if (c < H) {
      v = row[c];
    } else {
      v = 0.f;
      for (int t = 0; t < T; ++t) v += row[H + 1 + t] * mask[(long)t * ldm + (c - H)];
    }
    gW[(long)n * ldw + c] = v;
    if (c == 0 && gb) gb[n] = row[H];
  }
}

// Same product on a (column chunk, row) grid: no per-element 64-bit division (the grid-stride kernel above spent
// ~60 VALU per element on it and ran VALU-bound: 136 us for 256 x 360,022 at config 5), the row's T topology sums in
// registers; identical per-element arithmetic (bitwise equal).
template <int TT>
__global__ __launch_bounds__(256) void first_layer_grad_rows_kernel(const float* __restrict__ tmp, int N, int H, int T,
                                                                    int A, const float* __restrict__ mask, long ldm,
                                                                    float* __restrict__ gW, long ldw,
                                                                    float* __restrict__ gb) {
  const int n = blockIdx.y, W = H + A;
  const float* row = tmp + (long)n * (H + 1 + T);
  float r[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) r[t] = t < T ? row[H + 1 + t] : 0.f;
  float* g = gW + (long)n * ldw;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < W; c += gridDim.x * 256) {
    float v;
    if (c < H) {
      v = row[c];
    } else {
      v = 0.f;
#pragma unroll
      for (int t = 0; t < TT; ++t)
        if (t < T) v += r[t] * mask[(long)t * ldm + (c - H)];
    }
    g[c] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && gb) gb[n] = row[H];
}

// dst[r][c] = src[r][c] * colmask[c]  (bf16, strided source -> aligned dense copy)
__global__ __launch_bounds__(256) void copy2d_kernel(const __hip_bfloat16* src, long lds_, __hip_bfloat16* dst,
                                                     long ldd, int R, int C, const float* colmask) {
  const long total = (long)R * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i - (long)r * C);
    float v = __bfloat162float(src[(long)r * lds_ + c]);
    if (colmask) v *= colmask[c];
    dst[(long)r * ldd + c] = __float2bfloat16(v);
  }
}

// copy2d on a (column chunk, row) grid: no per-element 64-bit division (the grid-stride form above is VALU-bound on
// it: ~40 us per 64 x 360,000 block at config 5); four independent elements per thread and iteration
__global__ __launch_bounds__(256) void copy2d_rows_kernel(const __hip_bfloat16* __restrict__ src, long lds_,
                                                          __hip_bfloat16* __restrict__ dst, long ldd, int C,
                                                          const float* __restrict__ colmask) {
  const int r = blockIdx.y;
  const __hip_bfloat16* s = src + (long)r * lds_;
  __hip_bfloat16* d = dst + (long)r * ldd;
  const int step = gridDim.x * 1024;
  for (int c0 = blockIdx.x * 1024 + threadIdx.x; c0 < C; c0 += step) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 256 * j;
      v[j] = c < C ? __bfloat162float(s[c]) * (colmask ? colmask[c] : 1.f) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 256 * j;
      if (c < C) d[c] = __float2bfloat16(v[j]);
    }
  }
}

// dst[r][c] = bf16(src[r][c])
__global__ __launch_bounds__(256) void cast2d_kernel(const float* src, long lds_, __hip_bfloat16* dst, long ldd, int R,
                                                     int C) {
  const long total = (long)R * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i - (long)r * C);
    dst[(long)r * ldd + c] = __float2bfloat16(src[(long)r * lds_ + c]);
  }
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------
static int grid_for(long total, int cap = 4096) {
  long g = (total + 255) / 256;
  if (g > cap) g = cap;
  return g < 1 ? 1 : (int)g;
}

void head(uintptr_t h, long ldh, int B, int C, int mode, uintptr_t w, uintptr_t b, float gamma, uintptr_t r,
          uintptr_t d, uintptr_t y, uintptr_t dh, long lddh, uintptr_t part, int blocks, uintptr_t stream) {
  GSC_CHECK(C <= 256, "critic output layer input width must be <= 256");
  HeadArgs a{ptr<const __hip_bfloat16>(h), ldh, B, C, mode, ptr<const float>(w), ptr<const float>(b), gamma,
             1.f / (float)B, ptr<const float>(r), ptr<const float>(d), ptr<float>(y), ptr<__hip_bfloat16>(dh), lddh,
             ptr<float>(part)};
  const hipStream_t s = stream_of(stream);
  if (C <= 64) hipLaunchKernelGGL(head_kernel<1>, dim3(blocks), dim3(256), 0, s, a);
  else if (C <= 128) hipLaunchKernelGGL(head_kernel<2>, dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(head_kernel<4>, dim3(blocks), dim3(256), 0, s, a);
  check_launch();
}

void first_layer_grad(uintptr_t tmp, int N, int H, int T, int A, uintptr_t mask, long ldm, uintptr_t gW, long ldw,
                      uintptr_t gb, uintptr_t stream) {
  const char* fe = getenv("GSC_FLG_ROWS");  // 0: the grid-stride kernel (A/B)
  if (T <= 4 && N <= 65535 && !(fe && fe[0] == '0')) {
    const int cx = (int)std::min<long>(((long)H + A + 1023) / 1024, 4096);  // ~4 columns per thread
    hipLaunchKernelGGL(first_layer_grad_rows_kernel<4>, dim3((unsigned)std::max(cx, 1), (unsigned)N), dim3(256), 0,
                       stream_of(stream), ptr<const float>(tmp), N, H, T, A, ptr<const float>(mask), ldm, ptr<float>(gW),
                       ldw, ptr<float>(gb));
  } else {
    hipLaunchKernelGGL(first_layer_grad_kernel, dim3(grid_for((long)N * (H + A))), dim3(256), 0, stream_of(stream),
                       ptr<const float>(tmp), N, H, T, A, ptr<const float>(mask), ldm, ptr<float>(gW), ldw,
                       ptr<float>(gb));
  }
  check_launch();
}

void copy2d(uintptr_t src, long lds_, uintptr_t dst, long ldd, int R, int C, uintptr_t colmask, uintptr_t stream) {
  const char* ce = getenv("GSC_COPY2D_ROWS");  // 0: the grid-stride kernel (A/B)
  if (R <= 65535 && !(ce && ce[0] == '0')) {
    const int cx = std::max(1, std::min((C + 1023) / 1024, 4096));
    hipLaunchKernelGGL(copy2d_rows_kernel, dim3((unsigned)cx, (unsigned)R), dim3(256), 0, stream_of(stream),
                       ptr<const __hip_bfloat16>(src), lds_, ptr<__hip_bfloat16>(dst), ldd, C, ptr<const float>(colmask));
  } else {
    hipLaunchKernelGGL(copy2d_kernel, dim3(grid_for((long)R * C)), dim3(256), 0, stream_of(stream),
                       ptr<const __hip_bfloat16>(src), lds_, ptr<__hip_bfloat16>(dst), ldd, R, C,
                       ptr<const float>(colmask));
  }
  check_launch();
}
struct Cfg {
  int RM, RN, WM, WN;
};

template <int RM, int RN, int WM, int WN, int BK, bool A_COL, bool B_KN>
static void launch_cfg(const GemmArgs& g, int splits, hipStream_t s) {
  constexpr int BM = 32 * RM * WM, BN = 32 * RN * WN;
  dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN, splits);
  hipLaunchKernelGGL((gemm_kernel<RM, RN, WM, WN, BK, A_COL, B_KN>), grid, dim3(256), 0, s, g);
  check_launch();
}

// tile shapes: 0 = 128x128 (2x2 waves of 64x64), 1 = 128x64 (4x1 waves of 32x64), 2 = 64x64 (2x2 of 32x32),
// 3 = 64x128 (2x2 waves of 32x64); K staged BK = 32 or 64 deep per barrier
template <bool A_COL, bool B_KN, int BK>
static void launch_layout_bk(const GemmArgs& g, int tile, int splits, hipStream_t s) {
  switch (tile) {
    case 0: launch_cfg<2, 2, 2, 2, BK, A_COL, B_KN>(g, splits, s); break;
    case 1: launch_cfg<1, 2, 4, 1, BK, A_COL, B_KN>(g, splits, s); break;
    case 3: launch_cfg<1, 2, 2, 2, BK, A_COL, B_KN>(g, splits, s); break;
    default: launch_cfg<1, 1, 2, 2, BK, A_COL, B_KN>(g, splits, s); break;
  }
}
template <bool A_COL, bool B_KN>
static void launch_layout(const GemmArgs& g, int tile, int bk, int splits, hipStream_t s) {
  if (bk == 64) launch_layout_bk<A_COL, B_KN, 64>(g, tile, splits, s);
  else launch_layout_bk<A_COL, B_KN, 32>(g, tile, splits, s);
}

static Operand operand(uintptr_t p, long ld, int dtype) {
  Operand o;
  o.p = reinterpret_cast<const void*>(p);
  o.ld = ld;
  o.dtype = dtype;
  o.vec = dtype == DT_BF16 && (p % 16 == 0) && (ld % 8 == 0);
  o.vec32 = dtype == DT_F32 && (p % 16 == 0) && (ld % 4 == 0);
  o.rows = nullptr;
  return o;
}

// Python entry: every pointer is a raw device address (0 = absent).
void gemm(int layout, int M, int N, int K, uintptr_t a, long lda, int adt, uintptr_t b, long ldb, int bdt,
          py::dict ep, uintptr_t stream) {
  GemmArgs g{};
  g.a = operand(a, lda, adt);
  g.b = operand(b, ldb, bdt);
  g.M = M;
  g.N = N;
  g.K = K;
  if (ep.contains("a_rows")) g.a.rows = ptr<const int>(ep["a_rows"].cast<uintptr_t>());
  if (ep.contains("b_rows")) g.b.rows = ptr<const int>(ep["b_rows"].cast<uintptr_t>());
  g.aug_n0 = ep.contains("aug_n0") ? ep["aug_n0"].cast<int>() : -1;
  g.aug_t = ep.contains("aug_t") ? ep["aug_t"].cast<int>() : 0;
  g.aug_topo = ptr<const int>(ep.contains("aug_topo") ? ep["aug_topo"].cast<uintptr_t>() : 0);
  auto gp = [&](const char* k) -> uintptr_t { return ep.contains(k) ? ep[k].cast<uintptr_t>() : 0; };
  auto gl = [&](const char* k, long d) -> long { return ep.contains(k) ? ep[k].cast<long>() : d; };
  Epilogue& e = g.e;
  e.alpha = ep.contains("alpha") ? ep["alpha"].cast<float>() : 1.f;
  e.bias = ptr<const float>(gp("bias"));
  e.rowtab = ptr<const float>(gp("rowtab"));
  e.ld_rowtab = gl("ld_rowtab", N);
  e.topo = ptr<const int>(gp("topo"));
  e.colmask = ptr<const float>(gp("colmask"));
  e.ld_colmask = gl("ld_colmask", N);
  e.gate = ptr<const __hip_bfloat16>(gp("gate"));
  e.ld_gate = gl("ld_gate", N);
  e.rowscale = ptr<const float>(gp("rowscale"));
  e.gmul = ptr<const __hip_bfloat16>(gp("gmul"));
  e.ld_gmul = gl("ld_gmul", N);
  e.dsig = ptr<__hip_bfloat16>(gp("dsig"));
  e.ld_dsig = gl("ld_dsig", N);
  e.sigmoid = ep.contains("sigmoid") ? ep["sigmoid"].cast<int>() : 0;
  e.relu = ep.contains("relu") ? ep["relu"].cast<int>() : 0;
  e.clamp = ep.contains("clamp") ? 1 : 0;
  if (e.clamp) {
    py::tuple c = ep["clamp"].cast<py::tuple>();
    e.lo = c[0].cast<float>();
    e.hi = c[1].cast<float>();
  }
  e.accumulate = ep.contains("accumulate") ? ep["accumulate"].cast<int>() : 0;
  e.single_topo = ep.contains("single_topo") ? ep["single_topo"].cast<int>() : 0;
  e.c32 = ptr<float>(gp("c32"));
  e.ldc32 = gl("ldc32", N);
  e.c16 = ptr<__hip_bfloat16>(gp("c16"));
  e.ldc16 = gl("ldc16", N);
  e.vec16 = e.c16 && (gp("c16") % 16 == 0) && (e.ldc16 % 8 == 0);
  const int tile = ep.contains("tile") ? ep["tile"].cast<int>() : 0;
  int splits = ep.contains("splits") ? ep["splits"].cast<int>() : 1;
  const int BK = ep.contains("bk") && ep["bk"].cast<int>() == 64 ? 64 : 32;
  g.kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  if (g.kchunk < BK) g.kchunk = BK;
  splits = (K + g.kchunk - 1) / g.kchunk;
  if (splits < 1) splits = 1;
  g.slab = gl("slab", (long)M * e.ldc32);
  GSC_CHECK(splits == 1 || e.c32, "split-K needs c32 slabs");
  GSC_CHECK(!(e.rowtab || e.colmask) || e.topo, "rowtab/colmask need topo");
  GSC_CHECK(!(g.aug_n0 >= 0) || (layout == 1 || layout == 2), "aug columns need a B_KN operand");
  GSC_CHECK(!(e.accumulate && splits > 1), "accumulate with split-K: accumulate in splitk_reduce");
  GSC_CHECK(!(e.dsig && !e.sigmoid), "dsig needs the sigmoid epilogue");
  GSC_CHECK(splits == 1 || !(e.sigmoid || e.gmul), "sigmoid / gmul epilogues do not run with split-K");
  const hipStream_t s = stream_of(stream);
  switch (layout) {
    case 0: launch_layout<false, false>(g, tile, BK, splits, s); break;  // A_ROW, B_NK
    case 1: launch_layout<true, true>(g, tile, BK, splits, s); break;    // A_COL, B_KN (weight gradient)
    case 2: launch_layout<false, true>(g, tile, BK, splits, s); break;   // A_ROW, B_KN (input gradient)
    default: GSC_CHECK(false, "unknown gemm layout");
  }
}

int gemm_splits(int K, int splits, int bk) {
  const int BK = bk == 64 ? 64 : 32;
  int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  if (kchunk < BK) kchunk = BK;
  return (K + kchunk - 1) / kchunk;
}

void splitk_reduce(uintptr_t slabs, long slab, int splits, int M, int N, long lds_, uintptr_t out, long ldo,
                   float alpha, int accumulate, uintptr_t stream) {
  const long total = (long)M * N;
  long grid = (total + 63) / 64;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)grid), dim3(256), 0, stream_of(stream),
                     ptr<const float>(slabs), slab, splits, M, N, lds_, ptr<float>(out), ldo, alpha, accumulate);
  check_launch();
}

void cast2d(uintptr_t src, long lds_, uintptr_t dst, long ldd, int R, int C, uintptr_t stream) {
  hipLaunchKernelGGL(cast2d_kernel, dim3(grid_for((long)R * C)), dim3(256), 0, stream_of(stream), ptr<const float>(src),
                     lds_, ptr<__hip_bfloat16>(dst), ldd, R, C);
  check_launch();
}

// Bit-mask fold with 16-byte weight loads (the 4-byte pair loop above is latency-bound: ~106 us for a 256 x 360,000
// bf16 block that streams in ~25 us): the row is split at its first 16-byte-aligned element (rows are slices of a
// wider weight matrix, e.g. the first layer's mask block at column H), the aligned body goes 8 weights per lane per
// load with two loads in flight, the mask bits of those 8 weights come from one or two 32-bit words of the packed
// table; the few head / tail elements take the scalar path.  Same products, different fp32 summation order.
template <int TT>
__global__ __launch_bounds__(256) void rowdot_bits8_kernel(const uint32_t* __restrict__ xb, long ldx, int T,
                                                           const __hip_bfloat16* __restrict__ W, long ldw, int N,
                                                           int A, int achunk, float* out, long ldo) {
  __shared__ float red[4][TT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x, z = blockIdx.y;
  const int a0 = z * achunk, a1 = min(A, a0 + achunk);
  const __hip_bfloat16* wr = W + (long)n * ldw;
  const int mis = (int)((reinterpret_cast<uintptr_t>(wr + a0) >> 1) & 7);  // elements past a 16-byte boundary
  const int ab = min(a1, a0 + ((8 - mis) & 7));                            // first aligned element
  const int nv = (a1 - ab) >> 3;                                            // whole 8-element vectors
  const int ae = ab + 8 * nv;                                               // tail start
  float s[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) s[t] = 0.f;
  auto bits8 = [&](int t, int a) -> uint32_t {  // mask bits of elements a .. a + 7 (bit e = element a + e)
    const uint32_t* row = xb + (long)t * ldx;
    const int w = a >> 5, sh = a & 31;
    uint32_t v = row[w] >> sh;
    if (sh > 24) v |= row[w + 1] << (32 - sh);
    return v & 0xffu;
  };
  auto acc8 = [&](const uint4& q, int a) {
    const uint32_t u[4] = {q.x, q.y, q.z, q.w};
    float wv8[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wv8[2 * e] = __uint_as_float(u[e] << 16);
      wv8[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      if (t >= T) continue;
      const uint32_t b = bits8(t, a);
      float v = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) v += ((b >> e) & 1u) ? wv8[e] : 0.f;
      s[t] += v;
    }
  };
  // aligned body: vectors tid, tid + 256, ... four loads in flight
  int k = threadIdx.x;
  for (; k + 768 < nv; k += 1024) {
    uint4 q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = *reinterpret_cast<const uint4*>(wr + ab + 8 * (k + 256 * j));
#pragma unroll
    for (int j = 0; j < 4; ++j) acc8(q[j], ab + 8 * (k + 256 * j));
  }
  for (; k < nv; k += 256) acc8(*reinterpret_cast<const uint4*>(wr + ab + 8 * k), ab + 8 * k);
  // head [a0, ab) and tail [ae, a1): at most 7 elements each
  const int h = threadIdx.x;
  int a = h < ab - a0 ? a0 + h : (h - (ab - a0) < a1 - ae ? ae + h - (ab - a0) : -1);
  if (h >= 16) a = -1;
  if (a >= 0) {
    const float w0 = __bfloat162float(wr[a]);
#pragma unroll
    for (int t = 0; t < TT; ++t)
      if (t < T) s[t] += ((xb[(long)t * ldx + (a >> 5)] >> (a & 31)) & 1u) ? w0 : 0.f;
  }
#pragma unroll
  for (int t = 0; t < TT; ++t) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s[t] += __shfl_xor(s[t], off);
    if (lane == 0) red[wv][t] = s[t];
  }
  __syncthreads();
  if ((int)threadIdx.x < TT && (int)threadIdx.x < T) {
    const int t = threadIdx.x;
    const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    if (gridDim.y == 1) out[(long)t * ldo + n] = v;
    else out[((long)z * T + t) * N + n] = v;  // partial slab z
  }
}

// ws (optional, >= S T N floats): A split over S workgroups per row when N alone gives a small grid.
void rowdot(uintptr_t x, long ldx, int T, uintptr_t W, long ldw, int N, int A, uintptr_t out, long ldo,
            uintptr_t stream, uintptr_t ws, long ws_floats, uintptr_t xbits, long ldb) {
  if ((long)T * N <= 0) return;
  int S = 1;
  if (ws) {
    S = (2048 + N - 1) / N;
    S = std::min(S, std::max(1, A / 2048));
    S = std::min(S, 64);
    while (S > 1 && (long)S * T * N > ws_floats) --S;
  }
  int achunk = (A + S - 1) / S;
  achunk = (achunk + 1) & ~1;
  S = (A + achunk - 1) / achunk;
  const bool bits = xbits != 0;
  const int pair = (W % 4 == 0) && (ldw % 2 == 0) && (A % 2 == 0) && (bits || ((x % 8 == 0) && (ldx % 2 == 0)));
  const hipStream_t s = stream_of(stream);
  float* dst = S > 1 ? ptr<float>(ws) : ptr<float>(out);
  const float* xs = bits ? ptr<const float>(xbits) : ptr<const float>(x);
  const long lx = bits ? ldb : ldx;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)N, (unsigned)S), dim3(256), 0, s, xs, lx, T,
                       ptr<const __hip_bfloat16>(W), ldw, N, A, achunk, pair, dst, ldo);
  };
  const char* ve = getenv("GSC_ROWDOT_VEC");  // 0: the 4-byte pair loop (A/B)
  const bool vec8_env = !(ve && ve[0] == '0');
  if (bits && T <= 4 && vec8_env) {  // 16-byte weight loads (rowdot_bits8_kernel)
    auto go8 = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)N, (unsigned)S), dim3(256), 0, s, ptr<const uint32_t>(xbits), ldb, T,
                         ptr<const __hip_bfloat16>(W), ldw, N, A, achunk, dst, ldo);
    };
    if (T <= 1) go8(rowdot_bits8_kernel<1>);
    else if (T <= 2) go8(rowdot_bits8_kernel<2>);
    else go8(rowdot_bits8_kernel<4>);
  } else if (bits) {
    if (T <= 1) go(rowdot_kernel<1, true>);
    else if (T <= 2) go(rowdot_kernel<2, true>);
    else if (T <= 4) go(rowdot_kernel<4, true>);
    else go(rowdot_kernel<8, true>);
  } else {
    if (T <= 1) go(rowdot_kernel<1, false>);
    else if (T <= 2) go(rowdot_kernel<2, false>);
    else if (T <= 4) go(rowdot_kernel<4, false>);
    else go(rowdot_kernel<8, false>);
  }
  check_launch();
  if (S > 1) splitk_reduce(ws, (long)T * N, S, T, N, N, out, ldo, 1.f, 0, stream);
}

void topo_expand(uintptr_t src, long lds_, uintptr_t dst, long ldd, int R, int C, int T, uintptr_t topo,
                 uintptr_t stream) {
  hipLaunchKernelGGL(topo_expand_kernel, dim3(grid_for((long)R * T * C)), dim3(256), 0, stream_of(stream),
                     ptr<const __hip_bfloat16>(src), lds_, ptr<__hip_bfloat16>(dst), ldd, R, C, T, ptr<const int>(topo));
  check_launch();
}

}  // namespace mlp

void register_mlp(py::module_& m) {
  m.def("gemm", &mlp::gemm, "bf16 MFMA GEMM with fused epilogue (layout 0: A[M,K] B[N,K]; 1: A[K,M] B[K,N]; "
                            "2: A[M,K] B[K,N])");
  m.def("gemm_splits", &mlp::gemm_splits, py::arg("K"), py::arg("splits"), py::arg("bk") = 32,
        "effective split-K count for K and a requested split count");
  m.def("splitk_reduce", &mlp::splitk_reduce, "deterministic sum of split-K fp32 slabs into a strided output");
  m.def("cast2d", &mlp::cast2d, "fp32 -> bf16 strided 2-D copy");
  m.def("rowdot", &mlp::rowdot, "out[t][n] = sum_a x[t][a] W[n][a] (mask fold of a first layer, small GEMVs)",
        py::arg("x"), py::arg("ldx"), py::arg("T"), py::arg("W"), py::arg("ldw"), py::arg("N"), py::arg("A"),
        py::arg("out"), py::arg("ldo"), py::arg("stream"), py::arg("ws") = 0, py::arg("ws_floats") = 0,
        py::arg("xbits") = 0, py::arg("ldb") = 0);
  m.def("topo_expand", &mlp::topo_expand, "dst[r][t C + c] = (topo[r] == t) src[r][c] (bf16 per-topology blocks)");
  m.def("mlp_head", &mlp::head, "critic output layer + TD target / critic loss / actor loss (fused)");
  m.def("first_layer_grad", &mlp::first_layer_grad, "first-layer weight/bias/mask-block gradient from the aug GEMM");
  m.def("copy2d", &mlp::copy2d, "bf16 strided 2-D copy with optional column mask");
}

}  // namespace gsc
