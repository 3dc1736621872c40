// Fused exploration noise + schedule post-processing (reference simple_ddpg.py:182-201, 338-395).
//
// One thread per (env, src, sfc, sf) slice of n_pad destination weights, held in registers. Noise
// comes from a counter-based Philox stream keyed by (seed, step), so results do not depend on
// launch shape.  The two threshold/normalise passes run in fp64 with left-to-right sums like the
// reference's Python floats.
#include <pybind11/pybind11.h>

#include "../common.h"
#include "../sim/philox.h"

namespace py = pybind11;

namespace gsc {

__device__ __forceinline__ double round10(double x) { return rint(x * 1e10) / 1e10; }

// One thread per (env, src, sfc, sf) slice; the slice (P <= 32 weights) lives in registers.
// Noise: one Philox4x32-10 draw per pair of weights (keyed by (seed, step, first index)), fp32
// Box-Muller (both outputs used).  The threshold/normalise passes stay fp64 with left-to-right sums.
template <int PM>
__global__ __launch_bounds__(64) void explore_postprocess_kernel(const float* __restrict__ mu,
                                                                 const float* __restrict__ mask,
                                                                 const long long* __restrict__ topo,
                                                                 float* __restrict__ out, int E, int A, int P,
                                                                 int warmup, float rand_mu, float rand_sigma,
                                                                 uint32_t seed, uint32_t step, double thr, int passes) {
  const int R = A / P;
  const long slice = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (slice >= (long)E * R) return;
  const long base = slice * P;
  // mask row: per env [E, A], or the env's topology row of a [T, A] table
  const float* mrow = topo ? mask + topo[slice / R] * (long)A + (slice % R) * P : mask + base;
  double w[PM];
#pragma unroll
  for (int i = 0; i < PM; i += 2) {
    if (i < P) {
      const Philox4 r = philox4x32_10(seed, step, (uint64_t)(base + i));
      const float u0 = (float)(r.v[0] >> 8) * (1.0f / 16777216.0f);  // [0, 1)
      const float u1 = (float)(r.v[1] >> 8) * (1.0f / 16777216.0f);
      float a0, a1;
      if (warmup) {
        a0 = u0 * mrow[i];
        a1 = i + 1 < P ? u1 * mrow[i + 1] : 0.f;
      } else {
        const float rad = sqrtf(-2.0f * __logf(1.0f - u0));  // 1 - u0 in (0, 1]
        float sn, cs;
        __sincosf(6.283185307179586f * u1, &sn, &cs);
        float s0 = 2.0f * mu[base + i] - 1.0f + rand_mu + rand_sigma * (rad * cs);
        a0 = 0.5f * (s0 + 1.0f);
        a0 = a0 < 0.f ? 0.f : (a0 > 1.f ? 1.f : a0);
        a1 = 0.f;
        if (i + 1 < P) {
          float s1 = 2.0f * mu[base + i + 1] - 1.0f + rand_mu + rand_sigma * (rad * sn);
          a1 = 0.5f * (s1 + 1.0f);
          a1 = a1 < 0.f ? 0.f : (a1 > 1.f ? 1.f : a1);
        }
      }
      w[i] = (double)a0;
      if (i + 1 < PM) w[i + 1] = (double)a1;
    }
  }
  const double acc = 1.4901161193847656e-08;  // sqrt(float64 eps)
  for (int pass = 0; pass < passes; ++pass) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < PM; ++i)
      if (i < P) {
        const double x = w[i] >= thr ? w[i] : 0.0;
        w[i] = x;
        s += x;
      }
    if (s == 0.0) {
      const double u = round10(1.0 / P);
#pragma unroll
      for (int i = 0; i < PM; ++i) w[i] = u;
    } else if (fabs(1.0 - s) > acc) {
#pragma unroll
      for (int i = 0; i < PM; ++i)
        if (i < P) w[i] = round10(w[i] / s);
    }
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < PM; ++i)
      if (i < P) s2 += w[i];
    const double r = 1.0 - s2;
    if (r != 0.0) {
      // first element that can absorb the residual (the last one otherwise)
      bool done = false;
#pragma unroll
      for (int i = 0; i < PM; ++i)
        if (i < P && !done && (i == P - 1 || w[i] + r >= 0)) {
          w[i] += r;
          done = true;
        }
    }
  }
#pragma unroll
  for (int i = 0; i < PM; ++i)
    if (i < P) out[base + i] = (float)w[i];
}

// Lane-parallel variant for n_pad <= 32 (the common case): 32 lanes per slice (one weight per lane,
// two slices per wave), fp64 sums by cross-lane reductions and the residual's target element by a
// ballot -- the serial kernel above is one latency-bound thread per slice.  Same noise stream; the
// fp64 sums associate differently (results agree to float32 rounding).
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
  double w = 0.0;
  if (on) {
    const int i0 = i & ~1;
    const Philox4 r = philox4x32_10(seed, step, (uint64_t)(base + i0));
    const float u0 = (float)(r.v[0] >> 8) * (1.0f / 16777216.0f);
    const float u1 = (float)(r.v[1] >> 8) * (1.0f / 16777216.0f);
    float a;
    if (warmup) {
      a = (i & 1 ? u1 : u0) * mrow[i];
    } else {
      const float rad = sqrtf(-2.0f * __logf(1.0f - u0));
      float sn, cs;
      __sincosf(6.283185307179586f * u1, &sn, &cs);
      const float sv = 2.0f * mu[base + i] - 1.0f + rand_mu + rand_sigma * (rad * (i & 1 ? sn : cs));
      a = 0.5f * (sv + 1.0f);
      a = a < 0.f ? 0.f : (a > 1.f ? 1.f : a);
    }
    w = (double)a;
  }
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

void explore_postprocess(uintptr_t mu, uintptr_t mask, uintptr_t topo, uintptr_t out, int E, int A, int P, int warmup, float rand_mu,
                         float rand_sigma, uint32_t seed, uint32_t step, double thr, int passes, uintptr_t stream) {
  GSC_CHECK(A % P == 0, "action dim must be a multiple of n_pad");
  const long slices = (long)E * (A / P);
  const int block = 64;
  const int grid = (int)((slices + block - 1) / block);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, stream_of(stream), ptr<const float>(mu),
                       ptr<const float>(mask), ptr<const long long>(topo), ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step,
                       thr, passes);
  };
  if (P <= 32) {
    const int sl_per_block = 8;
    hipLaunchKernelGGL(explore_postprocess_lanes_kernel, dim3((int)((slices + sl_per_block - 1) / sl_per_block)), dim3(256), 0,
                       stream_of(stream), ptr<const float>(mu), ptr<const float>(mask), ptr<const long long>(topo),
                       ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step, thr, passes);
  } else if (P <= 32) go(explore_postprocess_kernel<32>);
  else if (P <= 64) go(explore_postprocess_kernel<64>);
  else if (P <= 128) go(explore_postprocess_kernel<128>);
  else if (P <= 256) go(explore_postprocess_kernel<256>);
  else GSC_CHECK(false, "n_pad > 256 not supported by the exploration kernel");
  check_launch();
}

void register_explore(py::module_& m) {
  m.def("explore_postprocess", &explore_postprocess, "fused exploration + threshold/normalise (device)");
}

}  // namespace gsc
