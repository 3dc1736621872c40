// Device replay ring: transition insert + Philox index sampling + row gather (reference
// src/rlsp/agents/buffer.py:23-89, GraphReplayBuffer.add / sample).
//
// The ring cursor lives on the device (int64 state [pos, full, draws, -]) so insert and sample are
// plain kernels with fixed arguments: both run inside captured HIP graphs, and nothing is read back
// to the host.  Sampling follows the reference: uniform over the filled rows, and once the ring is
// full the row at the write cursor (the next one to be overwritten) is excluded:
//
//     full:  idx = (pos + 1 + u * (cap - 1) >> 32) % cap        not full:  idx = u * pos >> 32
//
// with u the 32-bit Philox4x32-10 word (key = (seed, "repl"), counter = (draw << 32) | b / 4, word
// b % 4) -- independent of launch shape, identical on the host path (CPU training, tests).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <tuple>
#include <vector>

#include "../common.h"
#include "../sim/philox.h"

namespace py = pybind11;

namespace gsc {

constexpr uint32_t kReplayKey1 = 0x7265706cu;  // "repl"

struct ReplayState {  // int64 x 4 on the device (and in checkpoints)
  long long pos, full, draws, pad;
};

GSC_HD int replay_index(uint32_t seed, long long draw, int b, long long pos, long long full, long long cap) {
  const Philox4 r = philox4x32_10(seed, kReplayKey1, ((uint64_t)draw << 32) | (uint32_t)(b >> 2));
  const uint64_t u = r.v[b & 3];
  if (full) return (int)((pos + 1 + (long long)((u * (uint64_t)(cap - 1)) >> 32)) % cap);
  return (int)((u * (uint64_t)pos) >> 32);
}

// ---- sample: every thread draws one index; the draw counter advances in a second kernel ---------
__global__ __launch_bounds__(256) void replay_index_kernel(const ReplayState* st, uint32_t seed, int B, long long cap,
                                                           int32_t* idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) idx[b] = replay_index(seed, st->draws, b, st->pos, st->full, cap);
}
__global__ void replay_draw_done_kernel(ReplayState* st) { st->draws += 1; }

// rows of `row_bytes` in granules of G bytes: dst[b] = src[idx[b]]
template <class G>
__global__ __launch_bounds__(256) void gather_rows_kernel(const char* __restrict__ src, char* __restrict__ dst,
                                                          const int32_t* __restrict__ idx, int B, long row_g) {
  const long total = (long)B * row_g;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / row_g, k = i - b * row_g;
    reinterpret_cast<G*>(dst)[i] = reinterpret_cast<const G*>(src)[(long)idx[b] * row_g + k];
  }
}

// ---- insert: E rows at the cursor (no wrap-around bookkeeping on the host) ----------------------
// kind 0: raw granule copy; 1: float32 -> bf16 (actions); 2: uint8 -> float32 (dones)
template <class G, int KIND>
__global__ __launch_bounds__(256) void insert_rows_kernel(const ReplayState* __restrict__ st, const char* __restrict__ src,
                                                          char* __restrict__ dst, int E, long row_n, long long cap) {
  const long long pos = st->pos;
  const long total = (long)E * row_n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long e = i / row_n, k = i - e * row_n;
    const long d = ((pos + e) % cap) * row_n + k;
    if constexpr (KIND == 0) reinterpret_cast<G*>(dst)[d] = reinterpret_cast<const G*>(src)[i];
    if constexpr (KIND == 1) reinterpret_cast<__bf16*>(dst)[d] = (__bf16)reinterpret_cast<const float*>(src)[i];
    if constexpr (KIND == 2) reinterpret_cast<float*>(dst)[d] = (float)reinterpret_cast<const uint8_t*>(src)[i];
  }
}

// ---- every column of a sample / insert in one launch ----------------------------------------------
// A column is a [rows, row_g granules] tensor; granules of gsz bytes (16/8/4/2/1).  Gather kinds:
// 0 copy, 3 int64 -> int32 (topology ids straight into the learner's int32 buffer).  Insert kinds as
// insert_rows_kernel (0 copy, 1 f32 -> bf16, 2 u8 -> f32); row_g counts elements for kinds 1 / 2.
constexpr int kMaxCols = 8;
struct RCol {
  const char* src;
  char* dst;
  long row_g;
  long drow_g;  // insert: destination row length in the same units (>= row_g; padded ring rows)
  int gsz, kind;
};
struct RCols {
  RCol c[kMaxCols];
  long start[kMaxCols + 1];  // prefix sums of rows * row_g (work items per column)
  int n;
};

__device__ __forceinline__ void copy_granule(const char* s, char* d, int gsz) {
  switch (gsz) {
    case 16: *reinterpret_cast<int4*>(d) = *reinterpret_cast<const int4*>(s); break;
    case 8: *reinterpret_cast<int2*>(d) = *reinterpret_cast<const int2*>(s); break;
    case 4: *reinterpret_cast<int*>(d) = *reinterpret_cast<const int*>(s); break;
    case 2: *reinterpret_cast<short*>(d) = *reinterpret_cast<const short*>(s); break;
    default: *d = *s; break;
  }
}

// One grid row (blockIdx.y) per column, a grid-stride loop over its rows x granules with the (row,
// granule) pair stepped incrementally: no per-element 64-bit division / modulo, and the granule width
// a compile-time type (a 1.5 GB syn200 action gather went through one division per 16 bytes).
template <class G, class F>
__device__ __forceinline__ void col_loop(long rows, long rg, F&& f) {
  const long total = rows * rg;
  const long S = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  long r = i / rg, k = i - r * rg;
  const long sr = S / rg, sk = S - sr * rg;
  for (; i < total; i += S) {
    f(r, k);
    k += sk;
    r += sr;
    if (k >= rg) { k -= rg; ++r; }
  }
}

template <class G>
__device__ __forceinline__ void gather_col(const RCol& col, const int32_t* __restrict__ idx, int B) {
  const G* __restrict__ src = reinterpret_cast<const G*>(col.src);
  G* __restrict__ dst = reinterpret_cast<G*>(col.dst);
  const long rg = col.row_g;
  col_loop<G>(B, rg, [&](long b, long k) { dst[b * rg + k] = src[(long)idx[b] * rg + k]; });
}

// dst_c[b] = src_c[idx[b]] for every column (blockIdx.y = column); block (0, 0) also advances the draw
// counter (the index kernel that consumed it has completed)
__global__ __launch_bounds__(256) void gather_cols_kernel(RCols cs, const int32_t* __restrict__ idx, int B,
                                                          ReplayState* st) {
  if (st != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) st->draws += 1;
  const RCol& col = cs.c[blockIdx.y];
  if (col.kind == 3) {
    const long long* src = reinterpret_cast<const long long*>(col.src);
    int32_t* dst = reinterpret_cast<int32_t*>(col.dst);
    col_loop<int>(B, 1, [&](long b, long) { dst[b] = (int32_t)src[idx[b]]; });
    return;
  }
  switch (col.gsz) {
    case 16: gather_col<int4>(col, idx, B); break;
    case 8: gather_col<int2>(col, idx, B); break;
    case 4: gather_col<int>(col, idx, B); break;
    case 2: gather_col<short>(col, idx, B); break;
    default: gather_col<char>(col, idx, B); break;
  }
}

// insert: source row e -> ring row (pos + e) mod cap (pos + e < 2 cap: one conditional subtract)
template <class G>
__device__ __forceinline__ void insert_col(const RCol& col, long long pos, long long cap, int E) {
  const G* __restrict__ src = reinterpret_cast<const G*>(col.src);
  G* __restrict__ dst = reinterpret_cast<G*>(col.dst);
  const long rg = col.row_g, dg = col.drow_g;
  col_loop<G>(E, rg, [&](long e, long k) {
    long r = pos + e;
    if (r >= cap) r -= cap;
    dst[r * dg + k] = src[e * rg + k];
  });
}

__global__ __launch_bounds__(256) void insert_cols_kernel(RCols cs, const ReplayState* __restrict__ st, long long cap,
                                                          int E) {
  const long long pos = st->pos;
  const RCol& col = cs.c[blockIdx.y];
  if (col.kind == 1 || col.kind == 2) {
    const long rg = col.row_g, dg = col.drow_g;
    col_loop<char>(E, rg, [&](long e, long k) {
      long r = pos + e;
      if (r >= cap) r -= cap;
      const long d = r * dg + k, j = e * rg + k;
      if (col.kind == 1) reinterpret_cast<__bf16*>(col.dst)[d] = (__bf16)reinterpret_cast<const float*>(col.src)[j];
      else reinterpret_cast<float*>(col.dst)[d] = (float)reinterpret_cast<const uint8_t*>(col.src)[j];
    });
    return;
  }
  switch (col.gsz) {
    case 16: insert_col<int4>(col, pos, cap, E); break;
    case 8: insert_col<int2>(col, pos, cap, E); break;
    case 4: insert_col<int>(col, pos, cap, E); break;
    case 2: insert_col<short>(col, pos, cap, E); break;
    default: insert_col<char>(col, pos, cap, E); break;
  }
}

__global__ void replay_advance_kernel(ReplayState* st, int E, long long cap) {
  const long long p = st->pos + E;
  if (p >= cap) st->full = 1;
  st->pos = p % cap;
}

static int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}
// blocks per column of the column kernels: ~4 granules per thread for the largest column, at most
// 16K blocks (the loop strides over the rest)
static int cols_grid(long most) {
  long g = (most + 1023) / 1024;
  return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

template <class F>
static void by_granule(long bytes, uintptr_t a, uintptr_t b, F&& f) {
  const uintptr_t al = a | b | (uintptr_t)bytes;
  if (al % 16 == 0) f(int4{}, bytes / 16);
  else if (al % 8 == 0) f(int2{}, bytes / 8);
  else if (al % 4 == 0) f(int{}, bytes / 4);
  else if (al % 2 == 0) f(short{}, bytes / 2);
  else f(char{}, bytes);
}

// ------------------------------------------------------------------------------------------------
// Host mirrors (CPU path): same index stream, same cursor semantics.
// ------------------------------------------------------------------------------------------------
static void host_indices(ReplayState* st, uint32_t seed, int B, long long cap, int32_t* idx) {
  for (int b = 0; b < B; ++b) idx[b] = replay_index(seed, st->draws, b, st->pos, st->full, cap);
  st->draws++;
}

// Launchers.  `device` selects the HIP kernels (pointers are device memory) or the host path.
void replay_sample_indices(bool device, uintptr_t state, uint32_t seed, int B, long long cap, uintptr_t idx,
                           uintptr_t stream) {
  if (!device) {
    host_indices(ptr<ReplayState>(state), seed, B, cap, ptr<int32_t>(idx));
    return;
  }
  hipLaunchKernelGGL(replay_index_kernel, dim3((B + 255) / 256), dim3(256), 0, stream_of(stream),
                     ptr<const ReplayState>(state), seed, B, cap, ptr<int32_t>(idx));
  hipLaunchKernelGGL(replay_draw_done_kernel, dim3(1), dim3(1), 0, stream_of(stream), ptr<ReplayState>(state));
  check_launch();
}

void replay_gather(bool device, uintptr_t src, uintptr_t dst, uintptr_t idx, int B, long row_bytes,
                   uintptr_t stream) {
  if (!device) {
    const int32_t* ix = ptr<int32_t>(idx);
    for (int b = 0; b < B; ++b)
      std::memcpy(ptr<char>(dst) + (long)b * row_bytes, ptr<char>(src) + (long)ix[b] * row_bytes, row_bytes);
    return;
  }
  by_granule(row_bytes, src, dst, [&](auto g, long row_g) {
    using G = decltype(g);
    hipLaunchKernelGGL(gather_rows_kernel<G>, dim3(grid_for((long)B * row_g)), dim3(256), 0, stream_of(stream),
                       ptr<const char>(src), ptr<char>(dst), ptr<const int32_t>(idx), B, row_g);
  });
  check_launch();
}

// kind as in insert_rows_kernel; row_n = elements per row (kind 0: bytes per row)
void replay_insert(bool device, uintptr_t state, uintptr_t src, uintptr_t dst, int E, long row_n, long long cap,
                   int kind, uintptr_t stream, long dst_row_n = 0) {
  const long drow = dst_row_n > 0 ? dst_row_n : row_n;
  if (!device) {
    const long long pos = ptr<ReplayState>(state)->pos;
    for (int e = 0; e < E; ++e) {
      const long r = (long)((pos + e) % cap);
      for (long k = 0; k < row_n; ++k) {
        const long i = (long)e * row_n + k, d = r * drow + k;
        if (kind == 0) ptr<char>(dst)[d] = ptr<const char>(src)[i];
        else if (kind == 1) {
          // round-to-nearest-even float -> bf16 (same as the device conversion)
          uint32_t u;
          std::memcpy(&u, ptr<const float>(src) + i, 4);
          const uint32_t lsb = (u >> 16) & 1u;
          const uint16_t h = (u & 0x7fffffffu) > 0x7f800000u ? (uint16_t)((u >> 16) | 0x40u)
                                                              : (uint16_t)((u + 0x7fffu + lsb) >> 16);
          ptr<uint16_t>(dst)[d] = h;
        } else if (kind == 2) ptr<float>(dst)[d] = (float)ptr<const uint8_t>(src)[i];
      }
    }
    return;
  }
  GSC_CHECK(drow == row_n, "replay_insert: padded rows only through replay_insert_cols");
  const hipStream_t s = stream_of(stream);
  if (kind == 0) {
    by_granule(row_n, src, dst, [&](auto g, long row_g) {
      using G = decltype(g);
      hipLaunchKernelGGL((insert_rows_kernel<G, 0>), dim3(grid_for((long)E * row_g)), dim3(256), 0, s,
                         ptr<const ReplayState>(state), ptr<const char>(src), ptr<char>(dst), E, row_g, cap);
    });
  } else if (kind == 1) {
    hipLaunchKernelGGL((insert_rows_kernel<char, 1>), dim3(grid_for((long)E * row_n)), dim3(256), 0, s,
                       ptr<const ReplayState>(state), ptr<const char>(src), ptr<char>(dst), E, row_n, cap);
  } else {
    hipLaunchKernelGGL((insert_rows_kernel<char, 2>), dim3(grid_for((long)E * row_n)), dim3(256), 0, s,
                       ptr<const ReplayState>(state), ptr<const char>(src), ptr<char>(dst), E, row_n, cap);
  }
  check_launch();
}

static int granule_of(long bytes, uintptr_t a, uintptr_t b) {
  const uintptr_t al = a | b | (uintptr_t)bytes;
  return al % 16 == 0 ? 16 : al % 8 == 0 ? 8 : al % 4 == 0 ? 4 : al % 2 == 0 ? 2 : 1;
}

// One sample: Philox indices (as replay_sample_indices) then every column gathered by one kernel.
// cols: (src, dst, row_bytes, kind) with kind 0 copy / 3 int64 -> int32 (row_bytes = 8).
void replay_sample_cols(bool device, uintptr_t state, uint32_t seed, int B, long long cap, uintptr_t idx,
                        const std::vector<std::tuple<uintptr_t, uintptr_t, long, int>>& cols, uintptr_t stream) {
  GSC_CHECK(!cols.empty() && (int)cols.size() <= kMaxCols, "replay_sample_cols: 1..8 columns");
  if (!device) {
    host_indices(ptr<ReplayState>(state), seed, B, cap, ptr<int32_t>(idx));
    const int32_t* ix = ptr<int32_t>(idx);
    for (const auto& c : cols) {
      const uintptr_t src = std::get<0>(c), dst = std::get<1>(c);
      const long rb = std::get<2>(c);
      for (int b = 0; b < B; ++b) {
        if (std::get<3>(c) == 3) ptr<int32_t>(dst)[b] = (int32_t)ptr<const long long>(src)[ix[b]];
        else std::memcpy(ptr<char>(dst) + (long)b * rb, ptr<char>(src) + (long)ix[b] * rb, rb);
      }
    }
    return;
  }
  RCols cs{};
  cs.n = (int)cols.size();
  cs.start[0] = 0;
  for (int i = 0; i < cs.n; ++i) {
    const auto& c = cols[i];
    RCol& r = cs.c[i];
    r.src = ptr<const char>(std::get<0>(c));
    r.dst = ptr<char>(std::get<1>(c));
    r.kind = std::get<3>(c);
    const long rb = std::get<2>(c);
    GSC_CHECK(r.kind == 0 || (r.kind == 3 && rb == 8), "replay_sample_cols: kind 0 or 3 (int64 rows)");
    r.gsz = r.kind == 3 ? 8 : granule_of(rb, std::get<0>(c), std::get<1>(c));
    r.row_g = rb / r.gsz;
    cs.start[i + 1] = cs.start[i] + (long)B * r.row_g;
  }
  const hipStream_t s = stream_of(stream);
  hipLaunchKernelGGL(replay_index_kernel, dim3((B + 255) / 256), dim3(256), 0, s, ptr<const ReplayState>(state), seed,
                     B, cap, ptr<int32_t>(idx));
  long most = 0;
  for (int i = 0; i < cs.n; ++i) most = std::max(most, cs.start[i + 1] - cs.start[i]);
  hipLaunchKernelGGL(gather_cols_kernel, dim3(cols_grid(most), cs.n), dim3(256), 0, s, cs, ptr<const int32_t>(idx), B,
                     ptr<ReplayState>(state));
  check_launch();
}

// One insert of E rows at the cursor for every column, then the cursor advance.
// cols: (src, dst, row_n, kind) as replay_insert.
void replay_insert_cols(bool device, uintptr_t state, int E, long long cap,
                        const std::vector<std::tuple<uintptr_t, uintptr_t, long, int, long>>& cols, uintptr_t stream);

void replay_advance(bool device, uintptr_t state, int E, long long cap, uintptr_t stream) {
  if (!device) {
    ReplayState* st = ptr<ReplayState>(state);
    const long long p = st->pos + E;
    if (p >= cap) st->full = 1;
    st->pos = p % cap;
    return;
  }
  hipLaunchKernelGGL(replay_advance_kernel, dim3(1), dim3(1), 0, stream_of(stream), ptr<ReplayState>(state), E, cap);
  check_launch();
}

// ---- trainer metrics: acc[0..3] += (sum succ, sum drop, sum return of finished episodes, finished) ----
__global__ __launch_bounds__(256) void step_metrics_kernel(const float* __restrict__ stats, int nstats,
                                                           const float* __restrict__ ep_return,
                                                           const uint8_t* __restrict__ done, int E, double* acc) {
  __shared__ double red[4][256];
  double v[4] = {0, 0, 0, 0};
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    v[0] += stats[(long)e * nstats];
    v[1] += stats[(long)e * nstats + 1];
    if (done[e]) { v[2] += ep_return[e]; v[3] += 1.0; }
  }
  for (int j = 0; j < 4; ++j) red[j][threadIdx.x] = v[j];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int j = 0; j < 4; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 4) acc[threadIdx.x] += red[threadIdx.x][0];
}

void step_metrics(bool device, uintptr_t stats, int nstats, uintptr_t ep_return, uintptr_t done, int E, uintptr_t acc,
                  uintptr_t stream) {
  if (!device) {
    double v[4] = {0, 0, 0, 0};
    for (int e = 0; e < E; ++e) {
      v[0] += ptr<const float>(stats)[(long)e * nstats];
      v[1] += ptr<const float>(stats)[(long)e * nstats + 1];
      if (ptr<const uint8_t>(done)[e]) { v[2] += ptr<const float>(ep_return)[e]; v[3] += 1.0; }
    }
    for (int j = 0; j < 4; ++j) ptr<double>(acc)[j] += v[j];
    return;
  }
  hipLaunchKernelGGL(step_metrics_kernel, dim3(1), dim3(256), 0, stream_of(stream), ptr<const float>(stats), nstats,
                     ptr<const float>(ep_return), ptr<const uint8_t>(done), E, ptr<double>(acc));
  check_launch();
}

// cols: (src, dst, row_n, kind, dst_row_n) -- dst_row_n: the ring's row length (0: = row_n; larger for
// ring rows padded to a 16-byte multiple, e.g. bf16 actions of A % 8 != 0 columns)
void replay_insert_cols(bool device, uintptr_t state, int E, long long cap,
                        const std::vector<std::tuple<uintptr_t, uintptr_t, long, int, long>>& cols, uintptr_t stream) {
  GSC_CHECK(!cols.empty() && (int)cols.size() <= kMaxCols, "replay_insert_cols: 1..8 columns");
  if (!device) {
    for (const auto& c : cols)
      replay_insert(false, state, std::get<0>(c), std::get<1>(c), E, std::get<2>(c), cap, std::get<3>(c), 0,
                    std::get<4>(c));
    replay_advance(false, state, E, cap, 0);
    return;
  }
  RCols cs{};
  cs.n = (int)cols.size();
  cs.start[0] = 0;
  for (int i = 0; i < cs.n; ++i) {
    const auto& c = cols[i];
    RCol& r = cs.c[i];
    r.src = ptr<const char>(std::get<0>(c));
    r.dst = ptr<char>(std::get<1>(c));
    r.kind = std::get<3>(c);
    const long rn = std::get<2>(c), drn = std::get<4>(c) > 0 ? std::get<4>(c) : rn;
    GSC_CHECK(r.kind >= 0 && r.kind <= 2 && drn >= rn, "replay_insert_cols: kind 0..2, dst rows >= src rows");
    r.gsz = r.kind == 0 ? granule_of(rn, std::get<0>(c), std::get<1>(c)) : 1;
    if (r.kind == 0) r.gsz = std::min(r.gsz, granule_of(drn, 0, 0));
    r.row_g = r.kind == 0 ? rn / r.gsz : rn;
    r.drow_g = r.kind == 0 ? drn / r.gsz : drn;
    cs.start[i + 1] = cs.start[i] + (long)E * r.row_g;
  }
  const hipStream_t s = stream_of(stream);
  GSC_CHECK(E <= cap, "replay_insert_cols: more rows than the ring holds");
  long most = 0;
  for (int i = 0; i < cs.n; ++i) most = std::max(most, cs.start[i + 1] - cs.start[i]);
  hipLaunchKernelGGL(insert_cols_kernel, dim3(cols_grid(most), cs.n), dim3(256), 0, s, cs,
                     ptr<const ReplayState>(state), cap, E);
  hipLaunchKernelGGL(replay_advance_kernel, dim3(1), dim3(1), 0, s, ptr<ReplayState>(state), E, cap);
  check_launch();
}

int replay_index_host(uint32_t seed, long long draw, int b, long long pos, long long full, long long cap) {
  return replay_index(seed, draw, b, pos, full, cap);
}

void register_replay(py::module_& m) {
  m.def("replay_sample_indices", &replay_sample_indices);
  m.def("replay_gather", &replay_gather);
  m.def("replay_insert", &replay_insert, py::arg("device"), py::arg("state"), py::arg("src"), py::arg("dst"),
        py::arg("E"), py::arg("row_n"), py::arg("cap"), py::arg("kind"), py::arg("stream"), py::arg("dst_row_n") = 0);
  m.def("replay_advance", &replay_advance);
  m.def("replay_sample_cols", &replay_sample_cols, "Philox indices + every column gathered in one kernel");
  m.def("replay_insert_cols", &replay_insert_cols, "every column inserted in one kernel + cursor advance");
  m.def("replay_index", &replay_index_host, "one sampled index (host; for tests)");
  m.def("step_metrics", &step_metrics, "trainer metric accumulators (succ, drop, finished return, finished)");
}

}  // namespace gsc
