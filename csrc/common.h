// Shared helpers for the native extension (HIP launch checks, pointer casts).
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <cstdint>

#define GSC_HIP_CHECK(expr)                                                                      \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess)                                                                        \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +     \
                               __FILE__ + ":" + std::to_string(__LINE__) + " in " #expr);       \
  } while (0)

#define GSC_CHECK(cond, msg)                                                     \
  do {                                                                           \
    if (!(cond)) throw std::runtime_error(std::string("gsc_amd native: ") + msg); \
  } while (0)

namespace gsc {
template <class T>
inline T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }
inline hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
inline void check_launch() { GSC_HIP_CHECK(hipGetLastError()); }
}  // namespace gsc
