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

// Cross-stream hand-off by stream memory operations: the command processor of the producing stream writes a
// 32-bit sequence number once the stream's preceding work is done, and the consuming stream's processor polls
// for it (>=) before its next packet.  Replaces an event record + barrier-packet wait on the act <-> simulator
// chain between two simulator kernels.  The word lives in signal memory (hipMallocSignalMemory), as the API
// requires; kernels keep their own acquire / release fences, so data written before the value is visible to
// the consumer's kernels.
static bool stream_values_supported() {
  int dev = 0, v = 0;
  GSC_HIP_CHECK(hipGetDevice(&dev));
  GSC_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev));
  return v != 0;
}
static uintptr_t alloc_signal_words(int n) {
  void* p = nullptr;
  GSC_HIP_CHECK(hipExtMallocWithFlags(&p, sizeof(uint32_t) * (size_t)n, hipMallocSignalMemory));
  GSC_HIP_CHECK(hipMemset(p, 0, sizeof(uint32_t) * (size_t)n));
  GSC_HIP_CHECK(hipDeviceSynchronize());
  return reinterpret_cast<uintptr_t>(p);
}
static void free_signal_words(uintptr_t p) { GSC_HIP_CHECK(hipFree(reinterpret_cast<void*>(p))); }
static void stream_write_value(uintptr_t stream, uintptr_t word, uint32_t value) {
  GSC_HIP_CHECK(hipStreamWriteValue32(stream_of(stream), reinterpret_cast<void*>(word), value, 0));
}
static void stream_wait_value(uintptr_t stream, uintptr_t word, uint32_t value) {
  GSC_HIP_CHECK(hipStreamWaitValue32(stream_of(stream), reinterpret_cast<void*>(word), value, hipStreamWaitValueGte,
                                     0xFFFFFFFFu));
}

void register_streams(py::module_& m) {
  m.def("stream_values_supported", &stream_values_supported);
  m.def("alloc_signal_words", &alloc_signal_words, "n zeroed 32-bit words of signal memory (device pointer)");
  m.def("free_signal_words", &free_signal_words);
  m.def("stream_write_value", &stream_write_value, "stream writes value to word after its preceding work");
  m.def("stream_wait_value", &stream_wait_value, "stream waits until word >= value");
  m.def("cu_probe", &cu_probe, "record the hardware CU of each workgroup");
  m.def("create_cu_masked_stream", &create_cu_masked_stream, "HIP stream restricted to the given CUs");
  m.def("destroy_stream", &destroy_stream);
  m.def("cu_count", &cu_count);
}

}  // namespace gsc
