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

// Cross-stream hand-off by sequence words in fine-grained device memory (system-scope atomics: visible across
// XCDs and queues).  The producing stream runs signal_word_kernel after its work (an ordinary dispatch, back-to-back with
// the kernel before it in its queue); the consuming stream runs wait_word_kernel, one lane polling the word
// (>=, wrap-safe) with s_sleep between reads, before its next kernel.  Replaces an event record + barrier-packet
// wait on the act <-> simulator chain (and HIP's stream memory operations, whose write is a separately
// scheduled kernel ~10 us after the producer's last one: profiles/handoff_ab.txt).  Kernel boundaries keep
// their acquire / release fences, so data written before the word is visible to the consumer's kernels.  Every
// wait ends: after timeout_ticks of the 100 MHz constant clock it sets err and exits.  err is a mapped host word
// the trainer reads at every step, with at most a few steps enqueued ahead of the GPU, so a timed-out hand-off
// fails the run within those steps; the replay data written after the timeout is invalid (the run is aborted).
// Streams sharing a hardware queue (GPU_MAX_HW_QUEUES = 4, more streams under RCCL) cannot deadlock here: each
// wait is submitted after its producer's signal in submission order, so a shared queue only serialises them.
static bool stream_values_supported() {
  int dev = 0, v = 0;
  GSC_HIP_CHECK(hipGetDevice(&dev));
  GSC_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev));
  return v != 0;
}
static uintptr_t alloc_signal_words(int n) {
  void* p = nullptr;
  GSC_HIP_CHECK(hipExtMallocWithFlags(&p, sizeof(uint32_t) * (size_t)n, hipDeviceMallocFinegrained));
  GSC_HIP_CHECK(hipMemset(p, 0, sizeof(uint32_t) * (size_t)n));
  GSC_HIP_CHECK(hipDeviceSynchronize());
  return reinterpret_cast<uintptr_t>(p);
}
static void free_signal_words(uintptr_t p) { GSC_HIP_CHECK(hipFree(reinterpret_cast<void*>(p))); }
// One zeroed 32-bit word of coherent, mapped host memory: (host pointer, device pointer).  The wait kernel's
// timeout flag lives here, so the trainer reads it every step with a plain load (no copy, no stream sync).
static py::tuple alloc_host_word() {
  void* h = nullptr;
  void* d = nullptr;
  GSC_HIP_CHECK(hipHostMalloc(&h, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
  *reinterpret_cast<volatile uint32_t*>(h) = 0u;
  GSC_HIP_CHECK(hipHostGetDevicePointer(&d, h, 0));
  return py::make_tuple(reinterpret_cast<uintptr_t>(h), reinterpret_cast<uintptr_t>(d));
}
static void free_host_word(uintptr_t h) { GSC_HIP_CHECK(hipHostFree(reinterpret_cast<void*>(h))); }

__global__ void signal_word_kernel(uint32_t* word, uint32_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void wait_word_kernel(uint32_t* word, uint32_t value, uint32_t* err, long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  while ((int)(__hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - value) < 0) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}
static void signal_word(uintptr_t stream, uintptr_t word, uint32_t value) {
  hipLaunchKernelGGL(signal_word_kernel, dim3(1), dim3(64), 0, stream_of(stream), ptr<uint32_t>(word), value);
  check_launch();
}
static void wait_word(uintptr_t stream, uintptr_t word, uint32_t value, uintptr_t err, double timeout_s) {
  hipLaunchKernelGGL(wait_word_kernel, dim3(1), dim3(64), 0, stream_of(stream), ptr<uint32_t>(word), value,
                     ptr<uint32_t>(err), (long long)(timeout_s * 1e8));
  check_launch();
}
static uint32_t read_word(uintptr_t word) {
  uint32_t v = 0;
  GSC_HIP_CHECK(hipMemcpy(&v, reinterpret_cast<void*>(word), sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

void register_streams(py::module_& m) {
  m.def("stream_values_supported", &stream_values_supported);
  m.def("alloc_signal_words", &alloc_signal_words, "n zeroed 32-bit words of fine-grained device memory");
  m.def("free_signal_words", &free_signal_words);
  m.def("alloc_host_word", &alloc_host_word, "(host ptr, device ptr) of a zeroed coherent mapped host word");
  m.def("free_host_word", &free_host_word);
  m.def("signal_word", &signal_word, "stream stores value to word after its preceding work");
  m.def("wait_word", &wait_word, "stream waits until word >= value (err |= 1 after timeout_s)");
  m.def("read_word", &read_word);
  m.def("cu_probe", &cu_probe, "record the hardware CU of each workgroup");
  m.def("create_cu_masked_stream", &create_cu_masked_stream, "HIP stream restricted to the given CUs");
  m.def("destroy_stream", &destroy_stream);
  m.def("cu_count", &cu_count);
}

}  // namespace gsc
