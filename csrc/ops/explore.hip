// Fused exploration noise + schedule post-processing (reference simple_ddpg.py:182-201, 338-395).
//
// One thread per (env, src, sfc, sf) slice of n_pad destination weights. Noise comes from a
// counter-based Philox stream keyed by (seed, step), so results do not depend on launch shape.
// The two threshold/normalise passes run in fp64 with left-to-right sums like the reference's
// Python floats; the slice is kept in a per-thread global scratch row (slices are <= 1 KB).
#include <pybind11/pybind11.h>

#include "../common.h"
#include "../sim/philox.h"

namespace py = pybind11;

namespace gsc {

__device__ __forceinline__ double round10(double x) { return rint(x * 1e10) / 1e10; }

__global__ __launch_bounds__(256) void explore_postprocess_kernel(const float* __restrict__ mu,
                                                                  const float* __restrict__ mask,
                                                                  float* __restrict__ out, double* __restrict__ work,
                                                                  int E, int A, int P, int warmup, float rand_mu,
                                                                  float rand_sigma, uint32_t seed, uint32_t step,
                                                                  double thr, int passes) {
  const int R = A / P;
  const long slice = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (slice >= (long)E * R) return;
  const long base = slice * P;
  double* w = work + base;
  for (int i = 0; i < P; ++i) {
    const long g = base + i;
    const Philox4 r = philox4x32_10(seed, step, (uint64_t)g);
    float a;
    if (warmup) {
      const float u = (float)((r.v[0] >> 8) * (1.0 / 16777216.0));
      a = u * mask[g];
    } else {
      const double u1 = 1.0 - u01_53(r.v[0], r.v[1]);
      const double u2 = u01_53(r.v[2], r.v[3]);
      const float z = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
      float s = 2.0f * mu[g] - 1.0f;
      s += rand_mu + rand_sigma * z;
      a = 0.5f * (s + 1.0f);
      a = a < 0.f ? 0.f : (a > 1.f ? 1.f : a);
    }
    w[i] = (double)a;
  }
  const double acc = 1.4901161193847656e-08;  // sqrt(float64 eps)
  for (int pass = 0; pass < passes; ++pass) {
    double s = 0.0;
    for (int i = 0; i < P; ++i) {
      const double x = w[i] >= thr ? w[i] : 0.0;
      w[i] = x;
      s += x;
    }
    if (s == 0.0) {
      const double u = round10(1.0 / P);
      for (int i = 0; i < P; ++i) w[i] = u;
    } else if (fabs(1.0 - s) > acc) {
      for (int i = 0; i < P; ++i) w[i] = round10(w[i] / s);
    }
    double s2 = 0.0;
    for (int i = 0; i < P; ++i) s2 += w[i];
    const double r = 1.0 - s2;
    if (r != 0.0) {
      int i = 0;
      while (i < P - 1 && w[i] + r < 0) ++i;
      w[i] += r;
    }
  }
  for (int i = 0; i < P; ++i) out[base + i] = (float)w[i];
}

void explore_postprocess(uintptr_t mu, uintptr_t mask, uintptr_t out, int E, int A, int P, int warmup, float rand_mu,
                         float rand_sigma, uint32_t seed, uint32_t step, double thr, int passes, uintptr_t stream) {
  GSC_CHECK(A % P == 0, "action dim must be a multiple of n_pad");
  static double* work = nullptr;
  static long work_elems = 0;
  const long need = (long)E * A;
  if (need > work_elems) {
    if (work) GSC_HIP_CHECK(hipFree(work));
    GSC_HIP_CHECK(hipMalloc(&work, sizeof(double) * need));
    work_elems = need;
  }
  const long slices = (long)E * (A / P);
  const int block = 256;
  const int grid = (int)((slices + block - 1) / block);
  hipLaunchKernelGGL(explore_postprocess_kernel, dim3(grid), dim3(block), 0, stream_of(stream), ptr<const float>(mu),
                     ptr<const float>(mask), ptr<float>(out), work, E, A, P, warmup, rand_mu, rand_sigma, seed, step,
                     thr, passes);
  check_launch();
}

void register_explore(py::module_& m) {
  m.def("explore_postprocess", &explore_postprocess, "fused exploration + threshold/normalise (device)");
}

}  // namespace gsc
