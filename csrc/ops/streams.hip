// CU-partitioned HIP streams: the simulator and the learner run concurrently on disjoint CU sets
// (hipExtStreamCreateWithCUMask), so the latency-bound simulator waves and the LDS-bandwidth-bound
// learner kernels do not compete for the same CUs' LDS and issue slots.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_ext.h>

#include <vector>

#include "../common.h"

namespace py = pybind11;

namespace gsc {

// mask: list of CU indices (0 .. cu_count-1) the stream may use.  Returns the hipStream_t handle.
static uintptr_t create_cu_masked_stream(std::vector<int> cus) {
  int dev = 0, n = 0;
  GSC_HIP_CHECK(hipGetDevice(&dev));
  GSC_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int c : cus) {
    GSC_CHECK(c >= 0 && c < n, "CU index out of range");
    mask[c / 32] |= 1u << (c % 32);
  }
  hipStream_t s = nullptr;
  GSC_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return reinterpret_cast<uintptr_t>(s);
}

static void destroy_stream(uintptr_t s) { GSC_HIP_CHECK(hipStreamDestroy(reinterpret_cast<hipStream_t>(s))); }

static int cu_count() {
  int dev = 0, n = 0;
  GSC_HIP_CHECK(hipGetDevice(&dev));
  GSC_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  return n;
}

// Records (xcc, se, cu) of every workgroup: out[blockIdx.x] = xcc << 16 | hw_id bits (cu, sh, se).
__global__ void cu_probe_kernel(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[blockIdx.x] = ((xcc & 0xf) << 16) | ((hw >> 8) & 0xffff);
    long t0 = clock64();
    while (clock64() - t0 < spin) {}
  }
}

static void cu_probe(uintptr_t out, int blocks, int spin, uintptr_t stream) {
  hipLaunchKernelGGL(cu_probe_kernel, dim3(blocks), dim3(64), 0, stream_of(stream), ptr<uint32_t>(out), spin);
  check_launch();
}

void register_streams(py::module_& m) {
  m.def("cu_probe", &cu_probe, "record the hardware CU of each workgroup");
  m.def("create_cu_masked_stream", &create_cu_masked_stream, "HIP stream restricted to the given CUs");
  m.def("destroy_stream", &destroy_stream);
  m.def("cu_count", &cu_count);
}

}  // namespace gsc
