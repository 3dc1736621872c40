// Counter-based Philox4x32-10 RNG (per-env key, per-draw counter) shared by host and device.
// Results are independent of how envs are distributed over GPUs / workgroups.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GSC_HD __host__ __device__ __forceinline__
// Handlers are force-inlined too: measured on MI355X, out-of-line handlers (kernel code 188 KB ->
// 50 KB) made dispatch ~50 % slower (call overhead + the header then has to live in LDS).
#define GSC_HD_CALL GSC_HD
#else
#define GSC_HD inline
#define GSC_HD_CALL inline
#endif

// Wave-uniform hint for handler control values (type, state, indices, branch conditions): the
// device handlers run in one lane, so every loaded value is technically per-lane; reading it back
// through readfirstlane puts it in an SGPR, which turns the exec-mask branch trees of a VGPR
// switch into scalar branches and moves index arithmetic to the scalar ALU.  Identity on the host.
#if defined(__HIP_DEVICE_COMPILE__)
#define GSC_UNI(x) __builtin_amdgcn_readfirstlane((int)(x))
#else
#define GSC_UNI(x) ((int)(x))
#endif

namespace gsc {

struct Philox4 {
  uint32_t v[4];
};

GSC_HD void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c0 = hi1 ^ c1 ^ k0;
  c1 = lo1;
  c2 = hi0 ^ c3 ^ k1;
  c3 = lo0;
}

// One 128-bit block for (key, 64-bit counter).
GSC_HD Philox4 philox4x32_10(uint32_t k0, uint32_t k1, uint64_t ctr) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x9E3779B9u, c3 = 0x243F6A88u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  Philox4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// 53-bit uniform in [0, 1) from two 32-bit words.
GSC_HD double u01_53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

}  // namespace gsc
