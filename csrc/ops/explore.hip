// Fused exploration noise + schedule post-processing (reference simple_ddpg.py:182-201, 338-395).
//
// Lane-parallel over each (env, src, sfc, sf) slice of n_pad destination weights: two slices per
// wave (32 lanes each) up to n_pad = 32, one slice per wave with up to four consecutive weights per
// lane up to n_pad = 256 (the 200-node configs).  Noise comes from a counter-based Philox stream keyed
// by (seed, step, flat quad index) -- one draw per four weights -- so results do not depend on launch
// shape.  The two
// threshold/normalise passes run in fp64 (cross-lane sums; the reference sums Python floats left to
// right, so results agree to float32 rounding) with the residual of the rounded sum added to the
// first weight that can absorb it, found by a ballot.
#include <pybind11/pybind11.h>

#include "../common.h"
#include "../sim/philox.h"

namespace py = pybind11;

namespace gsc {

// Round to 10 decimals: x * 1e10 to the nearest integer, scaled back by a multiply (1 ulp of fp64 from the
// division the reference's round(x, 10) implies; invisible after the float32 store)
__device__ __forceinline__ double round10(double x) { return rint(x * 1e10) * 1e-10; }

// Noise of the 4 weights of flat quad f4 (= flat index & ~3): ONE Philox4x32-10 draw keyed by (seed, step, f4),
// its four uniforms -> warm-up: the uniforms; else two fp32 Box-Muller pairs (v0, v1) -> weights 0, 1 and
// (v2, v3) -> weights 2, 3.  The value of a weight depends only on (seed, step, flat index).
struct Quad { float x[4]; };
__device__ __forceinline__ Quad explore_quad(uint64_t f4, int warmup, uint32_t seed, uint32_t step) {
  const Philox4 r = philox4x32_10(seed, step, f4);
  Quad q;
#pragma unroll
  for (int j = 0; j < 4; ++j) q.x[j] = (float)(r.v[j] >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  if (warmup) return q;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float rad = sqrtf(-2.0f * __logf(1.0f - q.x[2 * p]));  // 1 - u in (0, 1]
    float sn, cs;
    __sincosf(6.283185307179586f * q.x[2 * p + 1], &sn, &cs);
    q.x[2 * p] = rad * cs;
    q.x[2 * p + 1] = rad * sn;
  }
  return q;
}

// Weight from its noise value z (normal, or the warm-up uniform) and mu / mask.
__device__ __forceinline__ float explore_apply(float z, float mu, float m, int warmup, float rand_mu, float rand_sigma) {
  if (warmup) return z * m;
  const float sv = 2.0f * mu - 1.0f + rand_mu + rand_sigma * z;
  const float a = 0.5f * (sv + 1.0f);
  return a < 0.f ? 0.f : (a > 1.f ? 1.f : a);
}

// Noisy (or warm-up uniform) weight i of the slice starting at flat index base (explore_quad's value for it,
// with only its own Box-Muller pair evaluated).
__device__ __forceinline__ float explore_weight(const float* __restrict__ mu, const float* __restrict__ mrow, long base,
                                                int i, int warmup, float rand_mu, float rand_sigma, uint32_t seed,
                                                uint32_t step) {
  const uint64_t f = (uint64_t)(base + i);
  const Philox4 r = philox4x32_10(seed, step, f & ~3ull);
  const int j = (int)(f & 3);
  const uint32_t va = (j & 2) ? r.v[2] : r.v[0], vb = (j & 2) ? r.v[3] : r.v[1];
  const float u0 = (float)(va >> 8) * (1.0f / 16777216.0f), u1 = (float)(vb >> 8) * (1.0f / 16777216.0f);
  if (warmup) return ((j & 1) ? u1 : u0) * mrow[i];
  const float rad = sqrtf(-2.0f * __logf(1.0f - u0));
  float sn, cs;
  __sincosf(6.283185307179586f * u1, &sn, &cs);
  return explore_apply(rad * ((j & 1) ? sn : cs), mu[base + i], 0.f, 0, rand_mu, rand_sigma);
}

// n_pad <= 32: 32 lanes per slice (one weight per lane), two slices per wave.
__device__ __forceinline__ double half_sum(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

__global__ __launch_bounds__(256) void explore_postprocess_lanes_kernel(const float* __restrict__ mu,
                                                                       const float* __restrict__ mask,
                                                                       const long long* __restrict__ topo,
                                                                       float* __restrict__ out, int E, int A, int P,
                                                                       int warmup, float rand_mu, float rand_sigma,
                                                                       uint32_t seed, uint32_t step, double thr,
                                                                       int passes) {
  const int R = A / P;
  const long slice = (long)blockIdx.x * (blockDim.x >> 5) + (threadIdx.x >> 5);
  const int i = threadIdx.x & 31;
  if (slice >= (long)E * R) return;  // whole 32-lane halves exit together
  const long base = slice * P;
  const bool on = i < P;
  const float* mrow = topo ? mask + topo[slice / R] * (long)A + (slice % R) * P : mask + base;
  double w = on ? (double)explore_weight(mu, mrow, base, i, warmup, rand_mu, rand_sigma, seed, step) : 0.0;
  const double acc = 1.4901161193847656e-08;  // sqrt(float64 eps)
  const unsigned long long half_mask = (threadIdx.x & 32) ? 0xffffffff00000000ull : 0x00000000ffffffffull;
  const int half_base = threadIdx.x & 32;
  for (int pass = 0; pass < passes; ++pass) {
    w = on && w >= thr ? w : 0.0;
    const double s = half_sum(w);
    if (s == 0.0) w = on ? round10(1.0 / P) : 0.0;
    else if (fabs(1.0 - s) > acc && on) w = round10(w * (1.0 / s));
    const double r = 1.0 - half_sum(w);
    if (r != 0.0) {
      // first element that can absorb the residual (the last one otherwise)
      const unsigned long long b = __ballot(on && (i == P - 1 || w + r >= 0)) & half_mask;
      if (b != 0 && (__ffsll((long long)b) - 1 - half_base) == i) w += r;
    }
  }
  if (on) out[base + i] = (float)w;
}

// Sum over the wave, broadcast: DPP row shifts + row broadcasts (VALU latency) instead of six LDS-routed
// shuffles; a fixed order, so every lane and every launch gets the same bits
__device__ __forceinline__ double wave_sum(double v) {
#define GSC_DPP_ADDD(ctrl, rm)                                                           \
  {                                                                                      \
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), ctrl, rm, 0xF, false); \
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), ctrl, rm, 0xF, false); \
    v += __hiloint2double(hi, lo);                                                       \
  }
  GSC_DPP_ADDD(0x111, 0xF) GSC_DPP_ADDD(0x112, 0xF) GSC_DPP_ADDD(0x114, 0xF) GSC_DPP_ADDD(0x118, 0xF)
  GSC_DPP_ADDD(0x142, 0xA) GSC_DPP_ADDD(0x143, 0xC)
#undef GSC_DPP_ADDD
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63), __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// 32 < n_pad <= 256: one slice per wave, K <= 4 consecutive weights per lane (lane l holds weights
// K l .. K l + K - 1, so "the first weight that can absorb the residual" is the first lane of a
// ballot, then the first of its K).
// Optional simulator hand-off (PMask.base != 0): the positive-destination bitset of every post-processed row,
// written into the simulator state's pmask block (what sim_pmask_kernel would derive from the stored action
// block in a second HBM pass).  Row (src, c, sf) of env e -> 4 x u64 at base + e stride + 32 ((src Cd + c) Sd
// + sf); bit d = (weight d > 0 and mask d > 0), i.e. a positive weight on a real destination of the topology.
struct PMask {
  char* base;
  long stride;
  int C, F, Cd, Sd;
};

template <int K>
__global__ __launch_bounds__(256) void explore_postprocess_wave_kernel(const float* __restrict__ mu,
                                                                      const float* __restrict__ mask,
                                                                      const long long* __restrict__ topo,
                                                                      float* __restrict__ out, int E, int A, int P,
                                                                      int warmup, float rand_mu, float rand_sigma,
                                                                      uint32_t seed, uint32_t step, double thr,
                                                                      int passes, PMask pm) {
  const int R = A / P;
  const long slice = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (slice >= (long)E * R) return;  // whole waves exit together
  const long base = slice * P;
  const float* mrow = topo ? mask + topo[slice / R] * (long)A + (slice % R) * P : mask + base;
  // lane's weights: flat indices f0 .. f0 + K - 1, within one or two Philox quads
  double w[K];
  {
    const int i0 = K * lane;
    const uint64_t f0 = (uint64_t)(base + i0);
    const bool any = i0 < P;
    Quad qa{}, qb{};
    if (any) {
      qa = explore_quad(f0 & ~3ull, warmup, seed, step);
      const uint64_t fl = f0 + K - 1;
      if ((fl >> 2) != (f0 >> 2) && i0 + (int)(((f0 & ~3ull) + 4) - f0) < P)
        qb = explore_quad(fl & ~3ull, warmup, seed, step);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = i0 + k;
      const int j = (int)((f0 & 3) + k);  // 0..6: quad a below 4, quad b from 4
      float z = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (j == t) z = qa.x[t];
        if (j == t + 4) z = qb.x[t];
      }
      w[k] = i < P ? (double)explore_apply(z, warmup ? 0.f : mu[base + i], warmup ? mrow[i] : 0.f, warmup, rand_mu,
                                           rand_sigma)
                   : 0.0;
    }
  }
  const double acc = 1.4901161193847656e-08;  // sqrt(float64 eps)
  const double uni = round10(1.0 / P);
  for (int pass = 0; pass < passes; ++pass) {
    double ps = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      w[k] = K * lane + k < P && w[k] >= thr ? w[k] : 0.0;
      ps += w[k];
    }
    const double s = wave_sum(ps);
    const bool renorm = fabs(1.0 - s) > acc;
    const double inv = s != 0.0 ? 1.0 / s : 0.0;  // one division per slice and pass
    ps = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool on = K * lane + k < P;
      if (s == 0.0) w[k] = on ? uni : 0.0;
      else if (renorm && on) w[k] = round10(w[k] * inv);
      ps += w[k];
    }
    const double r = 1.0 - wave_sum(ps);
    if (r != 0.0) {
      int first = -1;  // this lane's first weight that can absorb the residual
#pragma unroll
      for (int k = K - 1; k >= 0; --k) {
        const int i = K * lane + k;
        if (i < P && (i == P - 1 || w[k] + r >= 0)) first = k;
      }
      const unsigned long long b = __ballot(first >= 0);
      if (b != 0 && __ffsll((long long)b) - 1 == lane) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (k == first) w[k] += r;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (K * lane + k < P) out[base + K * lane + k] = (float)w[k];
  if (pm.base) {
    uint64_t bk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = K * lane + k;
      bk[k] = (uint64_t)__ballot(i < P && w[k] > 0.0 && mrow[i] > 0.f);
    }
    // destination d = K l + k sits at bit l of bk[k]: regroup into 64-destination words (lane q keeps word q)
    uint64_t word = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 64 * q + lane;
      const int kk = d % K, l = d / K;
      uint64_t b = bk[0];
#pragma unroll
      for (int k = 1; k < K; ++k)
        if (kk == k) b = bk[k];
      const uint64_t wq = (uint64_t)__ballot(d < P && ((b >> (l & 63)) & 1ull) && l < 64);
      if (lane == q) word = wq;
    }
    const int row = (int)(slice % R);
    const int sf = row % pm.F, c = (row / pm.F) % pm.C, src = row / (pm.F * pm.C);
    uint64_t* dst = reinterpret_cast<uint64_t*>(pm.base + (slice / R) * pm.stride) + 4L * ((src * pm.Cd + c) * pm.Sd + sf);
    if (lane < 4) dst[lane] = word;
  }
}

void explore_postprocess(uintptr_t mu, uintptr_t mask, uintptr_t topo, uintptr_t out, int E, int A, int P, int warmup, float rand_mu,
                         float rand_sigma, uint32_t seed, uint32_t step, double thr, int passes, uintptr_t stream,
                         py::object pmask) {
  GSC_CHECK(A % P == 0, "action dim must be a multiple of n_pad");
  GSC_CHECK(P <= 256, "n_pad > 256 not supported by the exploration kernel");
  PMask pm{nullptr, 0, 1, 1, 1, 1};
  if (!pmask.is_none()) {  // (base, stride, C, F, Cd, Sd)
    py::tuple t = pmask.cast<py::tuple>();
    pm.base = ptr<char>(t[0].cast<uintptr_t>());
    pm.stride = t[1].cast<long>();
    pm.C = t[2].cast<int>();
    pm.F = t[3].cast<int>();
    pm.Cd = t[4].cast<int>();
    pm.Sd = t[5].cast<int>();
    GSC_CHECK(P > 32 && (long)P * P * pm.C * pm.F == A && pm.C <= pm.Cd && pm.F <= pm.Sd,
              "explore pmask hand-off: n_pad > 32 and A = n_pad^2 C F within the simulator dims");
  }
  const long slices = (long)E * (A / P);
  if (P <= 32) {
    const int sl_per_block = 8;
    hipLaunchKernelGGL(explore_postprocess_lanes_kernel, dim3((int)((slices + sl_per_block - 1) / sl_per_block)), dim3(256), 0,
                       stream_of(stream), ptr<const float>(mu), ptr<const float>(mask), ptr<const long long>(topo),
                       ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step, thr, passes);
  } else {
    const int grid = (int)((slices + 3) / 4);  // four slices (waves) per block
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, stream_of(stream), ptr<const float>(mu), ptr<const float>(mask),
                         ptr<const long long>(topo), ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step, thr,
                         passes, pm);
    };
    if (P <= 64) go(explore_postprocess_wave_kernel<1>);
    else if (P <= 128) go(explore_postprocess_wave_kernel<2>);
    else if (P <= 192 && P % 2 == 1) go(explore_postprocess_wave_kernel<3>);
    else go(explore_postprocess_wave_kernel<4>);
  }
  check_launch();
}

void register_explore(py::module_& m) {
  m.def("explore_postprocess", &explore_postprocess, "fused exploration + threshold/normalise (device)",
        py::arg("mu"), py::arg("mask"), py::arg("topo"), py::arg("out"), py::arg("E"), py::arg("A"), py::arg("P"),
        py::arg("warmup"), py::arg("rand_mu"), py::arg("rand_sigma"), py::arg("seed"), py::arg("step"), py::arg("thr"),
        py::arg("passes"), py::arg("stream"), py::arg("pmask") = py::none());
}

}  // namespace gsc
