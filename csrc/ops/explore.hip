// Fused exploration noise + schedule post-processing (reference simple_ddpg.py:182-201, 338-395).
//
// Lane-parallel over each (env, src, sfc, sf) slice of n_pad destination weights: two slices per wave (32 lanes
// each) up to n_pad = 32; one slice per wave with up to four consecutive weights per lane up to n_pad = 128; two
// slices per wave with eight weights per lane above (the 200-node configs, n_pad % 8 == 0).  Noise comes from a
// counter-based Philox stream: above 32 destinations keyed by (seed, step, flat octet index) -- one draw per eight
// weights, 16-bit uniforms -- so results do not depend on which of those kernels runs; up to 32 the round-5 stream
// (one draw per quad, 24-bit uniforms, explore_weight).  The two threshold/normalise passes run in fp64
// (cross-lane sums; the reference sums Python floats left to right, so results agree to float32 rounding) with the
// residual of the rounded sum added to the first weight that can absorb it, found by a ballot.  Above 32
// destinations most rows skip them: when the second pass provably zeroes the whole row (FastExit), the kernel
// writes the uniform row directly, and its destination bitset from a per-topology table.
// At 200 nodes x 256 envs (92M weights): 565 -> 244 us noisy at round 5 (profiles/explore_r5.txt); round 6: raw
// hardware transcendentals, eight weights per draw, two slices per wave (profiles/explore_r6.txt).
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

// Box-Muller radius sqrt(-2 ln(1 - u0)) and (sin, cos)(2 pi u1) on the raw hardware transcendentals: v_log_f32
// (log2; 1 - u0 >= 2^-24 is never denormal), v_sqrt_f32 and v_sin / v_cos_f32 (argument in revolutions, so
// no 2 pi scaling).  The libm forms (__logf / sqrtf / __sincosf) add denormal scaling, an extended-precision
// ln 2 product and a sqrt correction step: ~35 VALU per pair instead of 8.
__device__ __forceinline__ float box_muller(float u0, float u1, float& sn, float& cs) {
  sn = __builtin_amdgcn_sinf(u1);
  cs = __builtin_amdgcn_cosf(u1);
  return __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(1.0f - u0));
}

// Philox4x32-10 round keys of (seed, step) computed once on the host: the wave kernel reads them from its
// arguments instead of bumping the key pair in every draw (20 scalar adds per wave).  Same bits as philox4x32_10.
struct RoundKeys {
  uint32_t k0[10], k1[10];
};
static RoundKeys round_keys(uint32_t k0, uint32_t k1) {
  RoundKeys rk;
  for (int r = 0; r < 10; ++r) {
    rk.k0[r] = k0;
    rk.k1[r] = k1;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return rk;
}
// a ^ b ^ k in ONE v_bitop3_b32 (truth table 0x96; the compiler does not form it from two xors): the round's two
// key mixes cost two VALU instead of four, 20 fewer per draw
__device__ __forceinline__ uint32_t xor3_k(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}
// philox4x32_10 (sim/philox.h) with the round keys from the host and the key mixes as xor3: same bits
__device__ __forceinline__ Philox4 philox_keyed(const RoundKeys& K, uint64_t ctr) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x9E3779B9u, c3 = 0x243F6A88u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    c0 = xor3_k((uint32_t)(p1 >> 32), c1, K.k0[r]);
    c1 = (uint32_t)p1;
    c2 = xor3_k((uint32_t)(p0 >> 32), c3, K.k1[r]);
    c3 = (uint32_t)p0;
  }
  Philox4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// Noise of flat octet o (weights 8o .. 8o + 7): ONE Philox4x32-10 draw keyed by (seed, step, o); its word p gives
// weights 8o + 2p (low 16 bits) and 8o + 2p + 1 (high 16 bits): in warm-up the two uniforms h 2^-16, else one
// Box-Muller pair (radius from the low half, angle from the high half; |z| <= 4.71, the 16-bit radius uniform's
// bound).  Eight weights per draw instead of four: the Philox rounds were half of the kernel's VALU issue.  The
// value of a weight depends only on (seed, step, flat index), whichever kernel computes it.
__device__ __forceinline__ void noise_pair(uint32_t w, int warmup, float& a, float& b) {
  const float u0 = (float)(w & 0xffffu) * (1.0f / 65536.0f), u1 = (float)(w >> 16) * (1.0f / 65536.0f);  // [0, 1)
  if (warmup) {
    a = u0;
    b = u1;
    return;
  }
  float sn, cs;
  const float rad = box_muller(u0, u1, sn, cs);
  a = rad * cs;
  b = rad * sn;
}

// The 4 weights of the 4-aligned quad f4: half of its octet's draw (words 0, 1 or 2, 3)
__device__ __forceinline__ Quad explore_quad(uint64_t f4, int warmup, const RoundKeys& rk) {
  const Philox4 r = philox_keyed(rk, f4 >> 3);
  const bool hi = (f4 & 4) != 0;
  Quad q;
  noise_pair(hi ? r.v[2] : r.v[0], warmup, q.x[0], q.x[1]);
  noise_pair(hi ? r.v[3] : r.v[1], warmup, q.x[2], q.x[3]);
  return q;
}

// Weight from its noise value z (normal, or the warm-up uniform) and mu / mask.
__device__ __forceinline__ float explore_apply(float z, float mu, float m, int warmup, float rand_mu, float rand_sigma) {
  if (warmup) return z * m;
  const float sv = 2.0f * mu - 1.0f + rand_mu + rand_sigma * z;
  // 0.5 (sv + 1) as fma(0.5, sv, 0.5): the same bits (scaling by 2 commutes with rounding), one VALU, and the clip
  // to [0, 1] folds into it as the clamp modifier
  return __builtin_amdgcn_fmed3f(__builtin_fmaf(0.5f, sv, 0.5f), 0.f, 1.f);
}

// Noisy (or warm-up uniform) weight i of the slice starting at flat index base, for the lanes kernel (n_pad <= 32,
// the Abilene-class configs): the round-5 stream, unchanged -- one Philox draw per 4-aligned quad of flat indices,
// 24-bit uniforms, libm Box-Muller.  The lanes kernel computes one draw per lane and weight either way, so the
// octet stream of the wider kernels would buy it nothing; keeping the stream keeps the headline config's action
// sequence (and hence its simulated traffic) what it was.
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

// Max over the wave of non-negative floats (lanes outside a DPP source read 0), same shift tree as wave_sum;
// compared as signed integers (order-preserving for non-negative floats, -0 counts as below 0), which folds
// the DPP into the max
__device__ __forceinline__ float wave_max_nonneg(float f) {
  int v = __float_as_int(f);
#define GSC_DPP_MAXI(ctrl, rm) v = max(v, __builtin_amdgcn_update_dpp(0, v, ctrl, rm, 0xF, false));
  GSC_DPP_MAXI(0x111, 0xF) GSC_DPP_MAXI(0x112, 0xF) GSC_DPP_MAXI(0x114, 0xF) GSC_DPP_MAXI(0x118, 0xF)
  GSC_DPP_MAXI(0x142, 0xA) GSC_DPP_MAXI(0x143, 0xC)
#undef GSC_DPP_MAXI
  return __int_as_float(max(__builtin_amdgcn_readlane(v, 63), 0));
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
  int ident;  // C == Cd and F == Sd: the bitset of action row r sits at 32 r bytes (no index split)
  int rows;   // action rows the simulator's block holds (N C F of its largest topology): rows past it (sources
              // >= N when n_pad > N) have no bitset and are skipped -- they would land in the next env's state
};

// Host-side constants of the early uniform exit (passes == 2, thr > 0): the rows whose second pass zeroes
// every weight -- at n_pad 50-200 nearly all of them (profiles/learning_curves.md, round 5) -- get the
// reference's all-zero answer, the uniform row, without the fp64 passes.  Pass 1's output is w / s rounded
// to 10 decimals plus a residual below 2e-8, so its largest entry is below thr - 1e-7 whenever the largest
// thresholded w is below (thr - 2e-7) s; the test runs on an fp32 sum of the same thresholded weights, with
// a 2^-11 relative margin that covers the fp32 sum's error (< 2e-5 for 256 terms).  Rows near the margin take
// the general fp64 loop.
struct FastExit {
  int on;         // passes == 2 and thr > 0
  float thr_f;    // smallest float f with (double) f >= thr: the fp32 threshold test selects the fp64 one's set
  double bound;   // (thr - 2e-7) (1 - 2^-11)
  int zero_ok;    // round10(1 / P) + 1e-7 < thr: an all-zero pass 1 (uniform row) is also zeroed by pass 2
  float uni, uni0;  // the uniform row: (float) round10(1 / P) and weight 0 with the residual
                    // 1 - (left-to-right sum of P copies), as normalize_scheduling_probabilities adds it
};

// Sum / max over the wave in fp32 (DPP folded into the add / max), same shift tree as wave_sum
__device__ __forceinline__ float wave_sum_f32(float v) {
#define GSC_DPP_ADDF(ctrl, rm) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, rm, 0xF, false));
  GSC_DPP_ADDF(0x111, 0xF) GSC_DPP_ADDF(0x112, 0xF) GSC_DPP_ADDF(0x114, 0xF) GSC_DPP_ADDF(0x118, 0xF)
  GSC_DPP_ADDF(0x142, 0xA) GSC_DPP_ADDF(0x143, 0xC)
#undef GSC_DPP_ADDF
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Lane's K raw noisy weights of one slice (undefined at and beyond P) from its K inputs v (mu, or the mask row in
// warm-up): flat indices f0 .. f0 + K - 1, within one or two Philox quads (one when vec: K = 4, 4-aligned rows)
template <int K>
__device__ __forceinline__ void explore_raw(float (&wf)[K], const float (&v)[K], long base, int i0, int P, bool vec,
                                            int warmup, float rand_mu, float rand_sigma, const RoundKeys& rk) {
  const uint64_t f0 = (uint64_t)(base + i0);
  const Quad qa = explore_quad(f0 & ~3ull, warmup, rk);  // lanes past P compute it too (no branch)
  Quad qb{};
  if (!vec) {
    const uint64_t fl = f0 + K - 1;
    if ((fl >> 2) != (f0 >> 2) && i0 + (int)(((f0 & ~3ull) + 4) - f0) < P) qb = explore_quad(fl & ~3ull, warmup, rk);
  }
  float z[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (vec) {  // f0 is 4-aligned (4-aligned rows, 4 weights per lane): weight k is quad entry k
      z[k] = qa.x[k & 3];
      continue;
    }
    const int j = (int)((f0 & 3) + k);  // 0..6: quad a below 4, quad b from 4
    z[k] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (j == t) z[k] = qa.x[t];
      if (j == t + 4) z[k] = qb.x[t];
    }
  }
  // one wave-uniform branch on warmup around the whole loop; weights past P are computed from the clamped
  // inputs and left in place (every consumer tests i < P), so there is no per-weight exec branch
  if (warmup) {
#pragma unroll
    for (int k = 0; k < K; ++k) wf[k] = explore_apply(z[k], 0.f, v[k], 1, rand_mu, rand_sigma);
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) wf[k] = explore_apply(z[k], v[k], 0.f, 0, rand_mu, rand_sigma);
  }
}

// Bitset word offset (in u64) of action row `row` in the simulator's pmask block of env `env`, or null for a
// row whose source node the simulator's block does not hold
__device__ __forceinline__ uint64_t* pmask_dst(const PMask& pm, int env, int row) {
  if (row >= pm.rows) return nullptr;  // rows are source-major: row >= N C F <=> source >= N
  long prow = row;
  if (!pm.ident) {
    const int sf = row % pm.F, c = (row / pm.F) % pm.C, sn = row / (pm.F * pm.C);
    prow = (long)(sn * pm.Cd + c) * pm.Sd + sf;
  }
  return reinterpret_cast<uint64_t*>(pm.base + env * pm.stride) + 4L * prow;
}

// General path of one slice: the reference's two fp64 threshold / normalise passes on the raw weights wf, the
// store, and the bitset from the final weights (rows the early exit does not decide; out of line, rare at
// 50-200 nodes)
template <int K>
__device__ __forceinline__ void explore_general(const float* __restrict__ mrow, float* __restrict__ out, long base,
                                             int P, int env, int row, int lane, double thr, int passes, PMask pm,
                                             float wf0, float wf1, float wf2, float wf3) {
  const float wf[4] = {wf0, wf1, wf2, wf3};
  double w[K];
#pragma unroll
  for (int k = 0; k < K; ++k) w[k] = (double)wf[k];
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
    uint64_t* dst = pmask_dst(pm, env, row);
    if (dst && lane < 4) dst[lane] = word;
  }
}

// S slices per wave (rows row0 .. row0 + S - 1 of env blockIdx.y), four waves per block: every input load of
// the S slices is issued up front (mu or mask row, and the mask words of the bitsets), the S Philox / reduction
// chains are independent (latency of one overlaps the other's), then each slice takes the early uniform exit or
// the general path.  env and rows come from the block index (scalar), no division.
template <int K, int S, bool VEC>
__global__ __launch_bounds__(256) void explore_postprocess_wave_kernel(const float* __restrict__ mu,
                                                                      const float* __restrict__ mask,
                                                                      const long long* __restrict__ topo,
                                                                      float* __restrict__ out, int E, int A, int P,
                                                                      int warmup, float rand_mu, float rand_sigma,
                                                                      uint32_t seed, uint32_t step, double thr,
                                                                      int passes, PMask pm, FastExit fx,
                                                                      RoundKeys rk) {
  const int R = A / P;
  const int row0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 * S + (threadIdx.x >> 6) * S));
  if (row0 >= R) return;  // whole waves exit together
  const int env = blockIdx.y, lane = threadIdx.x & 63, i0 = K * lane;
  constexpr bool vec = VEC;  // K = 4, 4-aligned rows, 16-byte aligned buffers: one 16-byte load / store per lane
  const float* mtab = topo ? mask + topo[env] * (long)A : mask + (long)env * A;  // [R, P] mask rows of this env
  float v[S][K], pmv[S][4], wf[S][K];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int row = min(row0 + s, R - 1);
    const long base = ((long)env * R + row) * P;
    const float* mrow = mtab + (long)row * P;
    const float* src = warmup ? mrow : mu + base;
    // loads from clamped (in-bounds) addresses, no exec-mask branch around them, and no use before the Philox
    // rounds (explore_raw zeroes the weights past P), so nothing waits for them early
    if (pm.base) {
#pragma unroll
      for (int q = 0; q < 4; ++q) pmv[s][q] = mrow[min(64 * q + lane, P - 1)];
    }
    if constexpr (VEC) {
      const float4 t = *reinterpret_cast<const float4*>(src + min(i0, P - 4));
      v[s][0] = t.x; v[s][K > 1 ? 1 : 0] = t.y; v[s][K > 2 ? 2 : 0] = t.z; v[s][K > 3 ? 3 : 0] = t.w;
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) v[s][k] = src[min(i0 + k, P - 1)];
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const long base = ((long)env * R + min(row0 + s, R - 1)) * P;
    explore_raw<K>(wf[s], v[s], base, i0, P, vec, warmup, rand_mu, rand_sigma, rk);
  }
  bool fast[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    fast[s] = false;
    if (fx.on) {
      float ps = 0.f, mx = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const bool keep = (i0 + k < P) & (wf[s][k] >= fx.thr_f);  // non-short-circuit: a select, not a branch
        const float t = keep ? wf[s][k] : 0.f;
        ps += t;
        mx = fmaxf(mx, t);
      }
      const float sum = wave_sum_f32(ps), M = wave_max_nonneg(mx);
      fast[s] = sum == 0.f ? fx.zero_ok != 0 : (double)M < fx.bound * (double)sum;
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int row = row0 + s;
    if (row >= R) break;
    const long base = ((long)env * R + row) * P;
    if (fast[s]) {
      if (vec) {
        if (i0 < P) *reinterpret_cast<float4*>(out + base + i0) = float4{lane == 0 ? fx.uni0 : fx.uni, fx.uni, fx.uni, fx.uni};
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (i0 + k < P) out[base + i0 + k] = lane == 0 && k == 0 ? fx.uni0 : fx.uni;
      }
      if (pm.base) {  // every weight is positive: the bitset is the topology's real destinations
        uint64_t word = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint64_t b = (uint64_t)__ballot(64 * q + lane < P && pmv[s][q] > 0.f);
          if (lane == q) word = b;
        }
        uint64_t* dst = pmask_dst(pm, env, row);
        if (dst && lane < 4) dst[lane] = word;
      }
    } else {
      explore_general<K>(mtab + (long)row * P, out, base, P, env, row, lane, thr, passes, pm, wf[s][0],
                         wf[s][K > 1 ? 1 : 0], wf[s][K > 2 ? 2 : 0], wf[s][K > 3 ? 3 : 0]);
    }
  }
}

// Sum / max over each 32-lane half of the wave (fp32, non-negative max as signed ints): DPP row shifts within the
// 16-lane rows, then row 0 -> 1 and row 2 -> 3 (row_bcast:15); the half totals end in lanes 31 and 63
__device__ __forceinline__ float half_sum_f32(float v) {
#define GSC_DPP_ADDF(ctrl, rm) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, rm, 0xF, false));
  GSC_DPP_ADDF(0x111, 0xF) GSC_DPP_ADDF(0x112, 0xF) GSC_DPP_ADDF(0x114, 0xF) GSC_DPP_ADDF(0x118, 0xF)
  GSC_DPP_ADDF(0x142, 0xA)
#undef GSC_DPP_ADDF
  return v;
}
__device__ __forceinline__ int half_max_i32(int v) {
#define GSC_DPP_MAXI(ctrl, rm) v = max(v, __builtin_amdgcn_update_dpp(0, v, ctrl, rm, 0xF, false));
  GSC_DPP_MAXI(0x111, 0xF) GSC_DPP_MAXI(0x112, 0xF) GSC_DPP_MAXI(0x114, 0xF) GSC_DPP_MAXI(0x118, 0xF)
  GSC_DPP_MAXI(0x142, 0xA)
#undef GSC_DPP_MAXI
  return v;
}

// 128 < n_pad <= 256, n_pad % 8 == 0 (the 200-node configs): TWO slices per wave, one per 32-lane half, eight
// consecutive weights per lane = one Philox draw per lane (explore_quad's noise, bit for bit) -- half the draws of
// the one-slice-per-wave kernel and half its per-slice reduction / address work.  Rows the early uniform exit
// decides are written from the host constants; their destination bitsets are the topology's real destinations,
// copied from the precomputed table pbits [T][R][4] (no mask loads, no ballots).  The rare other rows take the
// one-slice-per-wave path (four weights per lane: explore_raw + explore_general) for that row.
template <int WU, bool RM>  // RM: rand_mu != 0 (else its add is skipped: x + 0 == x for the non-negative-zero sums here)
__global__ __launch_bounds__(256) void explore_postprocess_oct_kernel(const float* __restrict__ mu,
                                                                     const float* __restrict__ mask,
                                                                     const long long* __restrict__ topo,
                                                                     float* __restrict__ out, int R, int P,
                                                                     float rand_mu, float rand_sigma, double thr,
                                                                     int passes, PMask pm, FastExit fx, RoundKeys rk,
                                                                     const uint64_t* __restrict__ pbits) {
  const int rowA = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 8 + (threadIdx.x >> 6) * 2));
  if (rowA >= R) return;  // whole waves exit together
  constexpr int warmup = WU;
  const int env = blockIdx.y, lane = threadIdx.x & 63, h = lane >> 5, i0 = 8 * (lane & 31);
  const long tp = topo ? topo[env] : (long)env;  // mask table row of this env
  const float* mtab = mask + tp * (long)R * P;
  const int row = min(rowA + h, R - 1);  // a half past R (R odd) recomputes row R - 1 and stores nothing
  const long base = ((long)env * R + row) * P;
  const float* src = warmup ? mtab + (long)row * P : mu + base;
  const float4 va = *reinterpret_cast<const float4*>(src + min(i0, P - 4));
  const float4 vb = *reinterpret_cast<const float4*>(src + min(i0 + 4, P - 4));
  const float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
  const Philox4 r = philox_keyed(rk, (uint64_t)(base + i0) >> 3);  // base + i0 is a multiple of 8 (P % 8 == 0)
  float wf[8];
#pragma unroll
  for (int p = 0; p < 4; ++p) noise_pair(r.v[p], warmup, wf[2 * p], wf[2 * p + 1]);
  if (warmup) {
#pragma unroll
    for (int k = 0; k < 8; ++k) wf[k] = explore_apply(wf[k], 0.f, v[k], 1, rand_mu, rand_sigma);
  } else {
    // explore_apply on weight pairs: 2 mu - 1 (+ rand_mu) + sigma z as packed FMAs (v_pk_fma_f32, the same
    // per-element IEEE operations), then fma(0.5, ., 0.5) with the clamp modifier per element: 4 VALU per pair
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      f2 sv = __builtin_elementwise_fma(f2{2.f, 2.f}, f2{v[2 * p], v[2 * p + 1]}, f2{-1.f, -1.f});
      if (RM) sv = sv + f2{rand_mu, rand_mu};
      sv = __builtin_elementwise_fma(f2{rand_sigma, rand_sigma}, f2{wf[2 * p], wf[2 * p + 1]}, sv);
      wf[2 * p] = __builtin_amdgcn_fmed3f(__builtin_fmaf(0.5f, sv.x, 0.5f), 0.f, 1.f);
      wf[2 * p + 1] = __builtin_amdgcn_fmed3f(__builtin_fmaf(0.5f, sv.y, 0.5f), 0.f, 1.f);
    }
  }
  bool fast0 = false, fast1 = false;
  if (fx.on) {
    float ps = 0.f, mx = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float t = wf[k] >= fx.thr_f ? wf[k] : 0.f;
      ps += t;
      mx = fmaxf(mx, t);
    }
    if (i0 >= P) ps = mx = 0.f;  // P % 8 == 0: a lane's 8 weights are all real or all padding
    const float sv = half_sum_f32(ps);
    const int mv = half_max_i32(__float_as_int(mx));
    const float s0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 31));
    const float s1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 63));
    const float m0 = __int_as_float(max(__builtin_amdgcn_readlane(mv, 31), 0));
    const float m1 = __int_as_float(max(__builtin_amdgcn_readlane(mv, 63), 0));
    fast0 = s0 == 0.f ? fx.zero_ok != 0 : (double)m0 < fx.bound * (double)s0;
    fast1 = s1 == 0.f ? fx.zero_ok != 0 : (double)m1 < fx.bound * (double)s1;
  }
  const bool mine = (h ? fast1 : fast0) && rowA + h < R;
  if (mine && i0 < P) {  // P % 8 == 0: all 8 weights of the lane are real
    float* o = out + base + i0;
    reinterpret_cast<float4*>(o)[0] = float4{i0 == 0 ? fx.uni0 : fx.uni, fx.uni, fx.uni, fx.uni};
    reinterpret_cast<float4*>(o)[1] = float4{fx.uni, fx.uni, fx.uni, fx.uni};
  }
  if (pm.base && mine && (lane & 31) < 4) {  // every weight is positive: the bitset is the topology's real destinations
    uint64_t* dst = pmask_dst(pm, env, row);
    if (dst) dst[lane & 31] = pbits[((long)tp * R + row) * 4 + (lane & 31)];
  }
  // rows the early exit does not decide: the whole wave, four weights per lane (the same noise bits)
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if ((hh ? fast1 : fast0) || rowA + hh >= R) continue;
    const int rw = rowA + hh;
    const long bw = ((long)env * R + rw) * P;
    const float* mrow = mtab + (long)rw * P;
    const float4 t = *reinterpret_cast<const float4*>((warmup ? mrow : mu + bw) + min(4 * lane, P - 4));
    const float v4[4] = {t.x, t.y, t.z, t.w};
    float w4[4];
    explore_raw<4>(w4, v4, bw, 4 * lane, P, true, warmup, rand_mu, rand_sigma, rk);
    explore_general<4>(mrow, out, bw, P, env, rw, lane, thr, passes, pm, w4[0], w4[1], w4[2], w4[3]);
  }
}

// Host constants of the early uniform exit (see FastExit)
static FastExit fast_exit(int P, double thr, int passes) {
  FastExit fx{};
  fx.on = passes == 2 && thr > 0.0;
  float f = (float)thr;
  if ((double)f < thr) f = nextafterf(f, INFINITY);
  while ((double)nextafterf(f, -INFINITY) >= thr) f = nextafterf(f, -INFINITY);
  fx.thr_f = f;
  fx.bound = (thr - 2e-7) * (1.0 - 1.0 / 2048.0);
  const double uni = std::nearbyint((1.0 / P) * 1e10) * 1e-10;  // round10, as on the device
  double sum = 0.0;
  for (int i = 0; i < P; ++i) sum += uni;  // left to right, as Python's sum()
  const double r = 1.0 - sum;
  fx.zero_ok = uni + 1e-7 < thr;
  fx.uni = (float)uni;
  fx.uni0 = (float)(uni + r);  // weight 0 absorbs the residual (uni + r >= 0)
  return fx;
}

void explore_postprocess(uintptr_t mu, uintptr_t mask, uintptr_t topo, uintptr_t out, int E, int A, int P, int warmup, float rand_mu,
                         float rand_sigma, uint32_t seed, uint32_t step, double thr, int passes, uintptr_t stream,
                         py::object pmask, uintptr_t pbits) {
  GSC_CHECK(A % P == 0, "action dim must be a multiple of n_pad");
  GSC_CHECK(P <= 256, "n_pad > 256 not supported by the exploration kernel");
  PMask pm{nullptr, 0, 1, 1, 1, 1, 1, 0};
  if (!pmask.is_none()) {  // (base, stride, C, F, Cd, Sd, N): N = source nodes of the simulator's pmask block
    py::tuple t = pmask.cast<py::tuple>();
    pm.base = ptr<char>(t[0].cast<uintptr_t>());
    pm.stride = t[1].cast<long>();
    pm.C = t[2].cast<int>();
    pm.F = t[3].cast<int>();
    pm.Cd = t[4].cast<int>();
    pm.Sd = t[5].cast<int>();
    GSC_CHECK(t.size() == 7, "explore pmask hand-off: (base, stride, C, F, Cd, Sd, N)");
    const int N = t[6].cast<int>();
    GSC_CHECK(P > 32 && (long)P * P * pm.C * pm.F == A && pm.C <= pm.Cd && pm.F <= pm.Sd && N >= 1 && N <= P,
              "explore pmask hand-off: n_pad > 32, A = n_pad^2 C F and N <= n_pad within the simulator dims");
    pm.rows = N * pm.C * pm.F;
    pm.ident = pm.C == pm.Cd && pm.F == pm.Sd;
  }
  const long slices = (long)E * (A / P);
  GSC_CHECK(slices < (1L << 31) - 4, "exploration: E * A / n_pad must fit in int32");
  if (P <= 32) {
    const int sl_per_block = 8;
    hipLaunchKernelGGL(explore_postprocess_lanes_kernel, dim3((int)((slices + sl_per_block - 1) / sl_per_block)), dim3(256), 0,
                       stream_of(stream), ptr<const float>(mu), ptr<const float>(mask), ptr<const long long>(topo),
                       ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step, thr, passes);
  } else {
    GSC_CHECK(E < 65536, "exploration: at most 65535 envs per launch");
    const FastExit fx = fast_exit(P, thr, passes);
    const RoundKeys rk = round_keys(seed, step);
    constexpr int S = 1;  // slices per wave (2 measured slower at 200 nodes: 278 vs 255 us, profiles/explore_r5.txt)
    const dim3 grid((unsigned)((A / P + 4 * S - 1) / (4 * S)), (unsigned)E);  // four waves per block
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream_of(stream), ptr<const float>(mu), ptr<const float>(mask),
                         ptr<const long long>(topo), ptr<float>(out), E, A, P, warmup, rand_mu, rand_sigma, seed, step, thr,
                         passes, pm, fx, rk);
    };
    const bool vec = P % 4 == 0 && mu % 16 == 0 && mask % 16 == 0 && out % 16 == 0;
    // two slices per wave, 8 weights per lane: 128 < n_pad, n_pad % 8 == 0, and with the bitset hand-off only
    // given the per-topology bitset table (GSC_EXPLORE_OCT=0: the one-slice-per-wave kernel)
    const char* oe = getenv("GSC_EXPLORE_OCT");
    const bool oct = P > 128 && P % 8 == 0 && vec && (!pm.base || (pbits && topo)) && !(oe && oe[0] == '0');
    if (oct) {
      const dim3 g8((unsigned)((A / P + 7) / 8), (unsigned)E);  // four waves x two slices per block
      auto* kern = warmup ? explore_postprocess_oct_kernel<1, false>
                          : (rand_mu != 0.f ? explore_postprocess_oct_kernel<0, true> : explore_postprocess_oct_kernel<0, false>);
      hipLaunchKernelGGL(kern, g8, dim3(256), 0,
                         stream_of(stream), ptr<const float>(mu), ptr<const float>(mask), ptr<const long long>(topo),
                         ptr<float>(out), A / P, P, rand_mu, rand_sigma, thr, passes, pm, fx, rk, ptr<const uint64_t>(pbits));
    } else if (P <= 64) go(explore_postprocess_wave_kernel<1, S, false>);
    else if (P <= 128) go(explore_postprocess_wave_kernel<2, S, false>);
    else if (P <= 192 && P % 2 == 1) go(explore_postprocess_wave_kernel<3, S, false>);
    else if (vec) go(explore_postprocess_wave_kernel<4, S, true>);
    else go(explore_postprocess_wave_kernel<4, S, false>);
  }
  check_launch();
}

void register_explore(py::module_& m) {
  m.def("explore_postprocess", &explore_postprocess, "fused exploration + threshold/normalise (device)",
        py::arg("mu"), py::arg("mask"), py::arg("topo"), py::arg("out"), py::arg("E"), py::arg("A"), py::arg("P"),
        py::arg("warmup"), py::arg("rand_mu"), py::arg("rand_sigma"), py::arg("seed"), py::arg("step"), py::arg("thr"),
        py::arg("passes"), py::arg("stream"), py::arg("pmask") = py::none(), py::arg("pbits") = 0);
}

}  // namespace gsc
