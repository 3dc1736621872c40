// Fused exploration noise + schedule post-processing (reference simple_ddpg.py:182-201, 338-395).
//
// Lane-parallel over each (env, src, sfc, sf) slice of n_pad destination weights: two slices per
// wave (32 lanes each) up to n_pad = 32, one slice per wave with up to four consecutive weights per
// lane up to n_pad = 256 (the 200-node configs).  Noise comes from a counter-based Philox stream keyed
// by (seed, step, weight index), so results do not depend on launch shape.  The two
// threshold/normalise passes run in fp64 (cross-lane sums; the reference sums Python floats left to
// right, so results agree to float32 rounding) with the residual of the rounded sum added to the
// first weight that can absorb it, found by a ballot.
#include <pybind11/pybind11.h>

#include "../common.h"
#include "../sim/philox.h"

namespace py = pybind11;

namespace gsc {

__device__ __forceinline__ double round10(double x) { return rint(x * 1e10) / 1e10; }

// Noisy (or warm-up uniform) weight i of the slice starting at flat index base: one Philox4x32-10
// draw per pair of weights (keyed by the pair's first index), fp32 Box-Muller, both outputs used.
__device__ __forceinline__ float explore_weight(const float* __restrict__ mu, const float* __restrict__ mrow, long base,
                                                int i, int warmup, float rand_mu, float rand_sigma, uint32_t seed,
                                                uint32_t step) {
  const int i0 = i & ~1;
  const Philox4 r = philox4x32_10(seed, step, (uint64_t)(base + i0));
  const float u0 = (float)(r.v[0] >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  const float u1 = (float)(r.v[1] >> 8) * (1.0f / 16777216.0f);
  if (warmup) return (i & 1 ? u1 : u0) * mrow[i];
  const float rad = sqrtf(-2.0f * __logf(1.0f - u0));  // 1 - u0 in (0, 1]
  float sn, cs;
  __sincosf(6.283185307179586f * u1, &sn, &cs);
  const float sv = 2.0f * mu[base + i] - 1.0f + rand_mu + rand_sigma * (rad * (i & 1 ? sn : cs));
  const float a = 0.5f * (sv + 1.0f);
  return a < 0.f ? 0.f : (a > 1.f ? 1.f : a);
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
    else if (fabs(1.0 - s) > acc && on) w = round10(w / s);
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

// Noisy (or warm-up uniform) weights i0, i0 + 1 of a slice from ONE Philox draw (the pair's two uniforms,
// both Box-Muller outputs) -- explore_weight's values for both members of the pair.
__device__ __forceinline__ void explore_pair(const float* __restrict__ mu, const float* __restrict__ mrow, long base,
                                            int i0, int warmup, float rand_mu, float rand_sigma, uint32_t seed,
                                            uint32_t step, float& w0, float& w1) {
  const Philox4 r = philox4x32_10(seed, step, (uint64_t)(base + i0));
  const float u0 = (float)(r.v[0] >> 8) * (1.0f / 16777216.0f);
  const float u1 = (float)(r.v[1] >> 8) * (1.0f / 16777216.0f);
  if (warmup) {
    w0 = u0 * mrow[i0];
    w1 = u1 * mrow[i0 + 1];
    return;
  }
  const float rad = sqrtf(-2.0f * __logf(1.0f - u0));
  float sn, cs;
  __sincosf(6.283185307179586f * u1, &sn, &cs);
  const float s0 = 2.0f * mu[base + i0] - 1.0f + rand_mu + rand_sigma * (rad * cs);
  const float s1 = 2.0f * mu[base + i0 + 1] - 1.0f + rand_mu + rand_sigma * (rad * sn);
  const float a0 = 0.5f * (s0 + 1.0f), a1 = 0.5f * (s1 + 1.0f);
  w0 = a0 < 0.f ? 0.f : (a0 > 1.f ? 1.f : a0);
  w1 = a1 < 0.f ? 0.f : (a1 > 1.f ? 1.f : a1);
}

// 32 < n_pad <= 256: one slice per wave, K <= 4 consecutive weights per lane (lane l holds weights
// K l .. K l + K - 1, so "the first weight that can absorb the residual" is the first lane of a
// ballot, then the first of its K).
template <int K>
__global__ __launch_bounds__(256) void explore_postprocess_wave_kernel(const float* __restrict__ mu,
                                                                      const float* __restrict__ mask,
                                                                      const long long* __restrict__ topo,
                                                                      float* __restrict__ out, int E, int A, int P,
                                                                      int warmup, float rand_mu, float rand_sigma,
                                                                      uint32_t seed, uint32_t step, double thr,
                                                                      int passes) {
  const int R = A / P;
  const long slice = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (slice >= (long)E * R) return;  // whole waves exit together
  const long base = slice * P;
  const float* mrow = topo ? mask + topo[slice / R] * (long)A + (slice % R) * P : mask + base;
  double w[K];
  if constexpr (K % 2 == 0) {  // K even: lanes own whole pairs (one Philox draw per pair)
#pragma unroll
    for (int k = 0; k < K; k += 2) {
      const int i = K * lane + k;
      float a = 0.f, b = 0.f;
      if (i + 1 < P) explore_pair(mu, mrow, base, i, warmup, rand_mu, rand_sigma, seed, step, a, b);
      else if (i < P) a = explore_weight(mu, mrow, base, i, warmup, rand_mu, rand_sigma, seed, step);  // odd P
      w[k] = a;
      w[k + 1] = b;
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = K * lane + k;
      w[k] = i < P ? (double)explore_weight(mu, mrow, base, i, warmup, rand_mu, rand_sigma, seed, step) : 0.0;
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
    ps = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool on = K * lane + k < P;
      if (s == 0.0) w[k] = on ? uni : 0.0;
      else if (renorm && on) w[k] = round10(w[k] / s);
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
}

void explore_postprocess(uintptr_t mu, uintptr_t mask, uintptr_t topo, uintptr_t out, int E, int A, int P, int warmup, float rand_mu,
                         float rand_sigma, uint32_t seed, uint32_t step, double thr, int passes, uintptr_t stream) {
  GSC_CHECK(A % P == 0, "action dim must be a multiple of n_pad");
  GSC_CHECK(P <= 256, "n_pad > 256 not supported by the exploration kernel");
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
                         passes);
    };
    if (P <= 64) go(explore_postprocess_wave_kernel<1>);
    else if (P <= 128) go(explore_postprocess_wave_kernel<2>);
    else if (P <= 192 && P % 2 == 1) go(explore_postprocess_wave_kernel<3>);
    else go(explore_postprocess_wave_kernel<4>);
  }
  check_launch();
}

void register_explore(py::module_& m) {
  m.def("explore_postprocess", &explore_postprocess, "fused exploration + threshold/normalise (device)");
}

}  // namespace gsc
