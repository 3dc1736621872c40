// Fused optimizer kernels over flat fp32 parameter buffers (reference: torch.optim.Adam defaults
// + Polyak soft target update, simple_ddpg.py:162-163, 229-234).
//
// adam_polyak: one pass reads (p, g, m, v, target) and writes (p, m, v, target):
//   m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v)/sqrt(bc2) + eps)          (torch's single-tensor Adam)
//   target = tau * p + (1 - tau) * target                     (after the step, as in the reference)
// The target update is fused because targets are only read by the *next* update.
// 16-byte vectorised, grid-stride; HBM-bound (20 B read + 16 B written per parameter).
#include <hip/hip_bf16.h>
#include <pybind11/pybind11.h>

#include "../common.h"

namespace py = pybind11;

namespace gsc {

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  float* target;  // may be null
  long n;
  float lr, b1, b2, eps, bc1, bc2_sqrt, tau, grad_scale, weight_decay;
  const long long* step;  // optional device step counter (HIP-graph replay); overrides bc1/bc2_sqrt
  const int* skip;        // optional device flag: non-zero -> leave p, m, v, target untouched (bad grads)
  __hip_bfloat16* p16;    // optional bf16 shadow of p (round-to-nearest-even, = autocast's cast)
  __hip_bfloat16* t16;    // optional bf16 shadow of target
};

__device__ __forceinline__ void store_bf16x4(__hip_bfloat16* dst, long i4, const float4& v) {
  __hip_bfloat16 h[4] = {__float2bfloat16(v.x), __float2bfloat16(v.y), __float2bfloat16(v.z), __float2bfloat16(v.w)};
  *reinterpret_cast<uint2*>(dst + 4 * i4) = *reinterpret_cast<const uint2*>(h);
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamArgs& a) {
  g *= a.grad_scale;
  if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, p, g);
  m = m + (1.f - a.b1) * (g - m);
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p - (a.lr / a.bc1) * (m / denom);
}

__global__ __launch_bounds__(256) void adam_polyak_kernel(AdamArgs a) {
  if (a.skip && *a.skip) return;
  if (a.step) {  // bias corrections from the device-resident step (same formulas as the host path)
    const double t = (double)*a.step;
    a.bc1 = (float)(1.0 - pow((double)a.b1, t));
    a.bc2_sqrt = (float)sqrt(1.0 - pow((double)a.b2, t));
  }
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    const float4 g = reinterpret_cast<const float4*>(a.g)[i];
    float4 m = reinterpret_cast<float4*>(a.m)[i];
    float4 v = reinterpret_cast<float4*>(a.v)[i];
    adam_one(p.x, g.x, m.x, v.x, a);
    adam_one(p.y, g.y, m.y, v.y, a);
    adam_one(p.z, g.z, m.z, v.z, a);
    adam_one(p.w, g.w, m.w, v.w, a);
    reinterpret_cast<float4*>(a.p)[i] = p;
    reinterpret_cast<float4*>(a.m)[i] = m;
    reinterpret_cast<float4*>(a.v)[i] = v;
    if (a.p16) store_bf16x4(a.p16, i, p);
    if (a.target) {
      float4 t = reinterpret_cast<float4*>(a.target)[i];
      t.x = a.tau * p.x + (1.f - a.tau) * t.x;
      t.y = a.tau * p.y + (1.f - a.tau) * t.y;
      t.z = a.tau * p.z + (1.f - a.tau) * t.z;
      t.w = a.tau * p.w + (1.f - a.tau) * t.w;
      reinterpret_cast<float4*>(a.target)[i] = t;
      if (a.t16) store_bf16x4(a.t16, i, t);
    }
  }
  // tail
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    float p = a.p[i], m = a.m[i], v = a.v[i];
    adam_one(p, a.g[i], m, v, a);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
    if (a.p16) a.p16[i] = __float2bfloat16(p);
    if (a.target) {
      a.target[i] = a.tau * p + (1.f - a.tau) * a.target[i];
      if (a.t16) a.t16[i] = __float2bfloat16(a.target[i]);
    }
  }
}

void adam_polyak(uintptr_t p, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t target, long n, float lr, float b1,
                 float b2, float eps, long step, float tau, float grad_scale, float weight_decay, uintptr_t stream,
                 uintptr_t step_ptr, uintptr_t skip_ptr, uintptr_t p16, uintptr_t t16) {
  GSC_CHECK((p & 15) == 0 && (g & 15) == 0 && (m & 15) == 0 && (v & 15) == 0 && (target & 15) == 0,
            "adam_polyak buffers must be 16-byte aligned");
  AdamArgs a;
  a.p = ptr<float>(p);
  a.g = ptr<const float>(g);
  a.m = ptr<float>(m);
  a.v = ptr<float>(v);
  a.target = target ? ptr<float>(target) : nullptr;
  a.n = n;
  a.lr = lr;
  a.b1 = b1;
  a.b2 = b2;
  a.eps = eps;
  a.bc1 = (float)(1.0 - pow((double)b1, (double)step));
  a.bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, (double)step));
  a.tau = tau;
  a.grad_scale = grad_scale;
  a.weight_decay = weight_decay;
  a.step = step_ptr ? ptr<const long long>(step_ptr) : nullptr;
  a.skip = skip_ptr ? ptr<const int>(skip_ptr) : nullptr;
  GSC_CHECK((p16 & 7) == 0 && (t16 & 7) == 0, "bf16 shadows must be 8-byte aligned");
  a.p16 = p16 ? ptr<__hip_bfloat16>(p16) : nullptr;
  a.t16 = t16 ? ptr<__hip_bfloat16>(t16) : nullptr;
  // ~2 float4 per thread: enough loads in flight to approach HBM bandwidth on the 90M-parameter actor of
  // the 200-node preset (the former 2,048-block cap left ~3.8 TB/s)
  const long n4 = (n + 3) / 4;
  long grid = (n4 + 511) / 512;
  if (grid > 65536) grid = 65536;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(adam_polyak_kernel, dim3((unsigned)grid), dim3(256), 0, stream_of(stream), a);
  check_launch();
}

__global__ __launch_bounds__(256) void polyak_kernel(float* __restrict__ t, const float* __restrict__ p, long n, float tau) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    t[i] = tau * p[i] + (1.f - tau) * t[i];
}

void polyak(uintptr_t target, uintptr_t p, long n, float tau, uintptr_t stream) {
  long grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(polyak_kernel, dim3((unsigned)(grid > 0 ? grid : 1)), dim3(256), 0, stream_of(stream),
                     ptr<float>(target), ptr<const float>(p), n, tau);
  check_launch();
}

// flag[0] = any non-finite value in g[0..n); flag[1] += flag[0] (skipped-update counter).
// One block per 64K elements, atomicOr into the flag; a second tiny launch bumps the counter.
// flag = [this step flagged, flagged-step count, bad-wave events (monotonic), events seen so far]:
// waves that see a non-finite gradient bump flag[2]; the single-thread kernel turns "flag[2] moved"
// into flag[0] -- no per-step memset (a runtime fill node in the captured update) is needed
__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ g, long n, int* flag) {
  int bad = 0;
  const long stride = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n4 = ((reinterpret_cast<uintptr_t>(g) & 15) == 0) ? n >> 2 : 0;  // 16-byte loads when aligned
  for (long i = t; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    bad |= !isfinite(v.x) | !isfinite(v.y) | !isfinite(v.z) | !isfinite(v.w);
  }
  for (long i = 4 * n4 + t; i < n; i += stride) bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(flag + 2, 1);
}
// flagged steps counter; optionally advances the device Adam step counter unless the step is skipped
__global__ void nonfinite_count_kernel(int* flag, long long* step) {
  const int bad = flag[2] != flag[3];
  flag[3] = flag[2];
  flag[0] = bad;
  flag[1] += bad;
  if (step && !bad) *step += 1;
}

void grad_guard(uintptr_t g, long n, uintptr_t flag, uintptr_t stream, uintptr_t step) {
  hipStream_t st = stream_of(stream);
  long grid = (n + 1023) / 1024;  // ~one float4 per thread
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)(grid > 0 ? grid : 1)), dim3(256), 0, st, ptr<const float>(g), n,
                     ptr<int>(flag));
  hipLaunchKernelGGL(nonfinite_count_kernel, dim3(1), dim3(1), 0, st, ptr<int>(flag), ptr<long long>(step));
  check_launch();
}

// ---- sharded optimizer (data parallel, ZeRO-1: gsc_amd/parallel/zero.py) ------------------------------
// local[0] = this rank's gradient shard holds a non-finite value (local[2]/[3]: monotonic event counters as
// in grad_guard); the ranks then agree on local[0] (all-reduce MAX) before guard_apply
__global__ void zflag_kernel(int* local) {
  local[0] = local[2] != local[3];
  local[3] = local[2];
}
void grad_guard_local(uintptr_t g, long n, uintptr_t local, uintptr_t stream) {
  hipStream_t st = stream_of(stream);
  long grid = (n + 1023) / 1024;
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)(grid > 0 ? grid : 1)), dim3(256), 0, st, ptr<const float>(g), n,
                     ptr<int>(local));
  hipLaunchKernelGGL(zflag_kernel, dim3(1), dim3(1), 0, st, ptr<int>(local));
  check_launch();
}
// the agreed flag -> the optimizer's guard (flag, flagged-step count) and the device Adam step counter
__global__ void guard_apply_kernel(const int* agreed, int* flag, long long* step) {
  const int bad = agreed[0] != 0;
  flag[0] = bad;
  flag[1] += bad;
  if (step && !bad) *step += 1;
}
void grad_guard_apply(uintptr_t agreed, uintptr_t flag, uintptr_t step, uintptr_t stream) {
  hipLaunchKernelGGL(guard_apply_kernel, dim3(1), dim3(1), 0, stream_of(stream), ptr<const int>(agreed), ptr<int>(flag),
                     ptr<long long>(step));
  check_launch();
}
// after the all-gather of the updated parameters: target = tau p + (1 - tau) target and both bf16 shadows
// over the whole buffer (skipped step: the target stays, the shadows are rewritten unchanged)
__global__ __launch_bounds__(256) void polyak_shadow_kernel(const float* __restrict__ p, float* __restrict__ t, long n,
                                                            float tau, __hip_bfloat16* p16, __hip_bfloat16* t16,
                                                            const int* skip) {
  const bool keep = skip && *skip;
  const long stride = (long)gridDim.x * blockDim.x;
  const long n4 = n >> 2;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 pv = reinterpret_cast<const float4*>(p)[i];
    if (p16) store_bf16x4(p16, i, pv);
    if (t) {
      float4 tv = reinterpret_cast<float4*>(t)[i];
      if (!keep) {
        tv.x = tau * pv.x + (1.f - tau) * tv.x;
        tv.y = tau * pv.y + (1.f - tau) * tv.y;
        tv.z = tau * pv.z + (1.f - tau) * tv.z;
        tv.w = tau * pv.w + (1.f - tau) * tv.w;
        reinterpret_cast<float4*>(t)[i] = tv;
      }
      if (t16) store_bf16x4(t16, i, tv);
    }
  }
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (p16) p16[i] = __float2bfloat16(p[i]);
    if (t) {
      if (!keep) t[i] = tau * p[i] + (1.f - tau) * t[i];
      if (t16) t16[i] = __float2bfloat16(t[i]);
    }
  }
}
void polyak_shadow(uintptr_t p, uintptr_t t, long n, float tau, uintptr_t p16, uintptr_t t16, uintptr_t skip,
                   uintptr_t stream) {
  GSC_CHECK((p & 15) == 0 && (t & 15) == 0 && (p16 & 7) == 0 && (t16 & 7) == 0, "polyak_shadow: aligned buffers");
  long grid = (n / 4 + 511) / 512;
  if (grid > 65536) grid = 65536;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(polyak_shadow_kernel, dim3((unsigned)grid), dim3(256), 0, stream_of(stream), ptr<const float>(p),
                     t ? ptr<float>(t) : nullptr, n, tau, p16 ? ptr<__hip_bfloat16>(p16) : nullptr,
                     t16 ? ptr<__hip_bfloat16>(t16) : nullptr, skip ? ptr<const int>(skip) : nullptr);
  check_launch();
}

void register_optim(py::module_& m) {
  m.def("grad_guard_local", &grad_guard_local, "local[0] = a non-finite value in this rank's gradient shard");
  m.def("grad_guard_apply", &grad_guard_apply, "guard flag / count / Adam step from the ranks' agreed flag");
  m.def("polyak_shadow", &polyak_shadow, "target Polyak update + bf16 shadows of params and target (full buffer)");
  m.def("grad_guard", &grad_guard, "flag[0] = any non-finite gradient; flag[1] counts flagged steps; step += !flag[0]",
        py::arg("g"), py::arg("n"), py::arg("flag"), py::arg("stream"), py::arg("step") = 0);
  m.def("adam_polyak", &adam_polyak, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("target"),
        py::arg("n"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("step"), py::arg("tau"),
        py::arg("grad_scale"), py::arg("weight_decay"), py::arg("stream"), py::arg("step_ptr") = 0,
        py::arg("skip_ptr") = 0, py::arg("p16") = 0, py::arg("t16") = 0);
  m.def("polyak", &polyak);
}

}  // namespace gsc
