// Batched simulator launchers: HIP kernels (one 64-lane wave per env) and the host path.
//
// Device mapping (CDNA4): each workgroup is one wave that owns one environment. The env's state
// blob is staged HBM -> LDS with 16-byte lane-strided copies, the discrete-event loop runs out of
// LDS (lane-parallel event selection over the pending-event array with a 6-step wave butterfly
// reduction; the handler itself is scalar in lane 0 — a DES is inherently sequential per env),
// and the blob is written back at the end of the 100 ms window. Thousands of envs give thousands
// of independent waves, which is what fills 256 CUs.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <thread>
#include <type_traits>
#include <vector>

#include "../common.h"
#include "sim_core.h"

namespace py = pybind11;

namespace gsc {

constexpr long kMaxEventsPerStep = 4000000;  // runaway guard (no GPU hang on a bad state)

struct SimArgs {
  char* states;
  long state_bytes;
  long lds_state_bytes;      // bytes of the blob staged in LDS (mode 1: all, mode 2: the hot prefix)
  Layout L;
  Dims D;
  SimConst K;
  const TopoDev* topos;
  const int32_t* topo_next;  // [E] topology used by the next reset of each env
  const uint32_t* seeds;     // [E]
  const float* actions;      // [E, action_stride]
  long action_stride;
  float* obs;                // [E, n_pad, n_obs]  obs for the next action (reset obs if done)
  float* next_obs;           // [E, n_pad, n_obs]  observation reached by this step (terminal if done)
  float* reward;             // [E]
  uint8_t* done;             // [E]
  float* stats;              // [E, kNumStats]
  float* ep_return;          // [E]  return of the episode that just finished (valid where done)
  int E;
  int use_lds;
  long topo_stage;           // bytes of LDS reserved for the staged topology tables
  unsigned long long* prof;  // optional [E, 4] cycle counters: select, dispatch, merge, events (diagnostic)
  int prio;                  // wave priority of the step kernel (s_setprio), see sim_step_kernel
  unsigned long long* prof_types;  // optional [E, 64, 2] dispatch cycles / count per (process type, state)
  int32_t* topo_cur;         // optional [E]: topology each env runs now (updated where an env was reset)
  int stage_pedges;          // the per-hop edge table is part of the staged topology
};

GSC_HD void step_epilogue(Env& S, const SimArgs& a, const SimConst& K, int env) {
  const TopoDev& T = a.topos[S.h->topo];
  const long ostride = (long)K.n_pad * K.n_obs;
  S.h->run_times++;
  finish_run_stats(S);
  const float r = compute_reward(S, K, T);
  write_stats(S, a.stats + (long)env * kNumStats);
  write_obs(S, K, T, a.next_obs + env * ostride);
  a.reward[env] = r;
  S.st->episode_return += r;
  S.h->run_count++;
  if (S.h->run_count >= K.episode_steps) {
    a.done[env] = 1;
    a.ep_return[env] = (float)S.st->episode_return;
    const int topo = a.topo_next[env];
    if (a.topo_cur) a.topo_cur[env] = topo;
    const int ep = S.h->episode + 1;
    env_init(S, K, a.topos[topo], topo, a.seeds[env], ep);
    write_obs(S, K, a.topos[topo], a.obs + env * ostride);
  } else {
    a.done[env] = 0;
    for (long i = 0; i < ostride; ++i) a.obs[env * ostride + i] = a.next_obs[env * ostride + i];
  }
}

GSC_HD void reset_one(Env& S, const SimArgs& a, int env) {
  const int topo = a.topo_next[env];
  S.st->episode_return = 0.0;
  S.st->ewma_flows = 1.0;
  env_init(S, a.K, a.topos[topo], topo, a.seeds[env], 1);
  write_obs(S, a.K, a.topos[topo], a.obs + (long)env * a.K.n_pad * a.K.n_obs);
}

// ------------------------------------------------------------------------------------------------
// Device path
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void copy16(char* dst, const char* src, long bytes, int lane) {
  const long n16 = bytes >> 4;
  for (long i = lane; i < n16; i += 64) reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(src)[i];
}

// write_obs with one node per lane: per-feature max by a wave butterfly (max is exact, so the
// values equal the serial host loop's), and optionally a second copy of the same observation.
__device__ __forceinline__ void write_obs_wave(const Env& S, const SimConst& K, int n, float* obs, float* obs2,
                                               int lane) {
  for (int j = 0; j < K.n_obs; ++j) {
    const int q = K.obs_feat[j];
    float mx = -__builtin_inff();
    for (int v = lane; v < n; v += 64) {
      const float x = obs_feature(S, K, q, v);
      mx = x > mx ? x : mx;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float o = __shfl_xor(mx, off);
      mx = o > mx ? o : mx;
    }
    const float den = mx + 1e-3f;
    for (int v = lane; v < K.n_pad; v += 64) {
      const float y = v < n ? clip01(obs_feature(S, K, q, v) / den) : 0.f;
      obs[v * K.n_obs + j] = y;
      if (obs2) obs2[v * K.n_obs + j] = y;
    }
  }
}

__device__ __forceinline__ int argmin_event_wave(const Env& S, int lane) {
  // the header copy is authoritative in lane 0 (the only lane that runs handlers)
  const int ne = __builtin_amdgcn_readfirstlane(S.h->n_events);
  double bt = 1e300;
  uint32_t bk = 0xffffffffu;
  int bi = -1;
  for (int i = lane; i < ne; i += 64) {
    const double t = S.events[i].t;
    const uint32_t k = S.events[i].key;
    if (t < bt || (t == bt && k < bk)) { bt = t; bk = k; bi = i; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ot = __shfl_xor(bt, off);
    const uint32_t ok = (uint32_t)__shfl_xor((int)bk, off);
    const int oi = __shfl_xor(bi, off);
    if (ot < bt || (ot == bt && ok < bk)) { bt = ot; bk = ok; bi = oi; }
  }
  return bi;
}

// Bytes of LDS used to stage SimConst + the env's topology tables in front of the state blob.
// (pedges: the per-hop edge and delay tables are staged too; else they are read from L2)
__host__ __device__ inline long topo_stage_bytes(const Dims& D, int H, bool pedges = true) {
  const long n2 = (long)D.N * D.N;
  return align16(sizeof(TopoDev)) + align16((int)(8 * D.N)) + align16((int)(8 * n2)) + align16((int)(2 * n2)) +
         (pedges ? 2 : 1) * align16((int)(2 * n2 * H)) + (pedges ? align16((int)(8 * n2 * H)) : 0) +
         align16((int)(2 * n2)) + align16((int)(8 * D.E)) + 2 * align16(2 * D.N);
}
__host__ __device__ inline long const_stage_bytes() { return align16(sizeof(SimConst)); }

// Copy one topology's tables into LDS and return a TopoDev whose pointers address the copies.
__device__ __forceinline__ TopoDev stage_topo(const TopoDev& g, char* dst, int lane, bool pedges) {
  TopoDev t = g;
  const int n = g.n, n2 = n * n;
  char* p = dst;
  auto put = [&](const void* src, int bytes) -> char* {
    char* d = p;
    const int w = bytes >> 1;  // 16-bit granules (every table is 2- or 8-byte typed)
    const int16_t* s16 = reinterpret_cast<const int16_t*>(src);
    int16_t* d16 = reinterpret_cast<int16_t*>(d);
    for (int i0 = 0; i0 < w; i0 += 64 * 8) {  // 8 loads in flight per lane (one HBM/L2 latency per 512 granules)
      int16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 64 * j + lane;
        v[j] = i < w ? s16[i] : (int16_t)0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 64 * j + lane;
        if (i < w) d16[i] = v[j];
      }
    }
    p += align16(bytes);
    return d;
  };
  t.cap = (const double*)put(g.cap, 8 * n);
  t.pdelay = (const double*)put(g.pdelay, 8 * n2);
  t.plen = (const int16_t*)put(g.plen, 2 * n2);
  t.pnodes = (const int16_t*)put(g.pnodes, 2 * n2 * g.H);
  if (pedges) {  // the per-hop edge and delay tables (else both are read from HBM / L2)
    t.pedges = (const int16_t*)put(g.pedges, 2 * n2 * g.H);
    t.phd = (const double*)put(g.phd, 8 * n2 * g.H);
  }
  t.edge_id = (const int16_t*)put(g.edge_id, 2 * n2);
  t.edge_cap = (const double*)put(g.edge_cap, 8 * (g.E > 0 ? g.E : 1));
  t.ingress = (const int16_t*)put(g.ingress, 2 * (g.n_ing > 0 ? g.n_ing : 1));
  t.egress = (const int16_t*)put(g.egress, 2 * (g.n_eg > 0 ? g.n_eg : 1));
  return t;
}

// ------------------------------------------------------------------------------------------------
// Sorted pending-event queue held in VGPRs across the wave: entry s*64+l lives in lane l, set s.
// pop = readfirstlane + DPP wave_shl:1, insert = ballot/popcount rank + DPP wave_shr:1 — no LDS.
// ------------------------------------------------------------------------------------------------
constexpr int DPP_WAVE_SHL1 = 0x130;
constexpr int DPP_WAVE_SHR1 = 0x138;

template <int QS>
struct RegQueue {
  uint32_t tlo[QS], thi[QS], key[QS];
  int32_t proc[QS];
  int n;
};

__device__ __forceinline__ double pack_t(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v, uint32_t lane0_in) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0_in, (int)v, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v, uint32_t lane63_in) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane63_in, (int)v, DPP_WAVE_SHL1, 0xF, 0xF, false);
}

template <int QS>
__device__ __forceinline__ void rq_init(RegQueue<QS>& q) {
#pragma unroll
  for (int s = 0; s < QS; ++s) { q.tlo[s] = 0xffffffffu; q.thi[s] = 0x7fefffffu; q.key[s] = 0xffffffffu; q.proc[s] = -1; }
  q.n = 0;
}

template <int QS>
__device__ __forceinline__ bool rq_insert(RegQueue<QS>& q, double t, uint32_t key, int proc, int lane) {
  if (q.n >= QS * 64) return false;
  int pos = 0;
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    if (s * 64 >= q.n) break;  // wave-uniform: only sets that hold entries
    const double et = pack_t(q.tlo[s], q.thi[s]);
    const bool less = (s * 64 + lane < q.n) && (et < t || (et == t && q.key[s] < key));
    pos += __popcll(__ballot(less));
  }
  const uint32_t tlo = (uint32_t)__double2loint(t), thi = (uint32_t)__double2hiint(t);
  // shift entries >= pos up by one, high set first (each set's carry is the previous set's lane 63)
#pragma unroll
  for (int s = QS - 1; s >= 0; --s) {
    if (s * 64 > q.n || (s + 1) * 64 <= pos) continue;  // set untouched by this insert
    const uint32_t c_tlo = s ? (uint32_t)__builtin_amdgcn_readlane((int)q.tlo[s - 1], 63) : 0u;
    const uint32_t c_thi = s ? (uint32_t)__builtin_amdgcn_readlane((int)q.thi[s - 1], 63) : 0u;
    const uint32_t c_key = s ? (uint32_t)__builtin_amdgcn_readlane((int)q.key[s - 1], 63) : 0u;
    const uint32_t c_prc = s ? (uint32_t)__builtin_amdgcn_readlane(q.proc[s - 1], 63) : 0u;
    const uint32_t sh_tlo = dpp_shr1(q.tlo[s], c_tlo), sh_thi = dpp_shr1(q.thi[s], c_thi);
    const uint32_t sh_key = dpp_shr1(q.key[s], c_key), sh_prc = dpp_shr1((uint32_t)q.proc[s], c_prc);
    const int idx = s * 64 + lane;
    if (idx > pos) { q.tlo[s] = sh_tlo; q.thi[s] = sh_thi; q.key[s] = sh_key; q.proc[s] = (int)sh_prc; }
    else if (idx == pos) { q.tlo[s] = tlo; q.thi[s] = thi; q.key[s] = key; q.proc[s] = proc; }
  }
  q.n++;
  return true;
}

template <int QS>
__device__ __forceinline__ void rq_pop(RegQueue<QS>& q, double& t, int& proc, uint32_t& key) {
  t = pack_t((uint32_t)__builtin_amdgcn_readfirstlane((int)q.tlo[0]), (uint32_t)__builtin_amdgcn_readfirstlane((int)q.thi[0]));
  proc = __builtin_amdgcn_readfirstlane(q.proc[0]);
  key = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.key[0]);
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    if (s * 64 >= q.n) break;  // remaining sets are empty
    const uint32_t c_tlo = s + 1 < QS ? (uint32_t)__builtin_amdgcn_readfirstlane((int)q.tlo[s + 1]) : 0xffffffffu;
    const uint32_t c_thi = s + 1 < QS ? (uint32_t)__builtin_amdgcn_readfirstlane((int)q.thi[s + 1]) : 0x7fefffffu;
    const uint32_t c_key = s + 1 < QS ? (uint32_t)__builtin_amdgcn_readfirstlane((int)q.key[s + 1]) : 0xffffffffu;
    const uint32_t c_prc = s + 1 < QS ? (uint32_t)__builtin_amdgcn_readfirstlane(q.proc[s + 1]) : 0xffffffffu;
    q.tlo[s] = dpp_shl1(q.tlo[s], c_tlo);
    q.thi[s] = dpp_shl1(q.thi[s], c_thi);
    q.key[s] = dpp_shl1(q.key[s], c_key);
    q.proc[s] = (int)dpp_shl1((uint32_t)q.proc[s], c_prc);
  }
  q.n--;
}

// Merge the events lane 0's handler appended to S.events (the inbox) into the register queue.
template <int QS>
__device__ __forceinline__ void rq_merge_inbox(RegQueue<QS>& q, Env& S, int lane) {
  const int nin = __builtin_amdgcn_readfirstlane(S.h->n_events);
  for (int i = 0; i < nin; ++i) {
    const Event e = S.events[i];
    if (!rq_insert(q, e.t, e.key, pack_target(e.proc, e.flow), lane)) S.h->flags |= FLAG_EVENT_OVERFLOW;
  }
  if (q.n > S.h->max_events) S.h->max_events = q.n;
  S.h->n_events = 0;
  __builtin_amdgcn_wave_barrier();
}

// Every lane runs the handlers on its own (identical) copy of the header and the same LDS state, so
// loaded values are wave-uniform and control flow stays scalar; loops over nodes / destinations
// inside a handler spread over the lanes (sim_core.h wave helpers).
// TLDS: the topology tables are staged in LDS (compile-time): every table pointer derives from the
// kernel's LDS array, so the handlers' table reads are ds_read (LDS address space) instead of flat
// loads through generic pointers (a runtime choice between an LDS copy and the HBM tables).
template <int QS, bool PROF, bool BIG, bool TLDS>
__device__ __forceinline__ void device_step_env(const SimArgs& a, const SimConst& K, char* base, char* topo_lds,
                                                int env, int lane, char* cold = nullptr) {
  const unsigned long long t_entry = PROF ? __builtin_amdgcn_s_memtime() : 0;
  Env S(base, a.L, a.D, cold);
  // Keep the env header in registers for the whole window (written back once at the end).
  Header* const h_mem = S.h;
  // (measured: header in LDS instead = 2.83 vs 2.30 ms/step for 256 Abilene envs)
  Header h_reg = *h_mem;
  S.h = &h_reg;
  if constexpr (BIG) S.act = a.actions + (long)env * a.action_stride;  // read in place of the schedule table
  const TopoDev T = [&] {
    if constexpr (TLDS) return stage_topo(a.topos[S.h->topo], topo_lds, lane, a.stage_pedges);
    else return a.topo_stage ? stage_topo(a.topos[S.h->topo], topo_lds, lane, a.stage_pedges) : a.topos[S.h->topo];
  }();
  load_action<BIG>(S, K, T, a.actions + (long)env * a.action_stride, lane, 64);
  __syncthreads();
  const unsigned long long t_act = PROF ? __builtin_amdgcn_s_memtime() : 0;
  // pending events -> sorted register queue; S.events then serves as the handlers' inbox
  RegQueue<QS> q;
  rq_init(q);
  rq_merge_inbox<QS>(q, S, lane);
  __syncthreads();  // every lane writes the same placement/sf tables: order the reads
  controller_prologue<BIG>(S, K, T);
  schedule_stop(S, K);
  __syncthreads();
  rq_merge_inbox<QS>(q, S, lane);
  constexpr bool prof = PROF;  // cycle counters compiled in only for the diagnostic variant
  unsigned long long t_sel = 0, t_hdl = 0, t_mrg = 0, n_ev = 0;
  const unsigned long long t_begin = prof ? __builtin_amdgcn_s_memtime() : 0;
  for (long it = 0;; ++it) {
    const unsigned long long t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    if (q.n <= 0 || it > kMaxEventsPerStep) {
      S.h->flags |= FLAG_BAD_STATE;
      break;
    }
    double et;
    int ep;
    uint32_t ek;
    rq_pop(q, et, ep, ek);
    const unsigned long long t1 = prof ? __builtin_amdgcn_s_memtime() : 0;
    if (target_proc(ep) == kStopProc) {
      S.h->now = et;
      break;
    }
    // Lane 0 runs the handler, then keeps going while the smallest event the handler chain just
    // scheduled precedes the queue head (lane 0 holds the head: entry 0 of set 0): those events
    // -- process initialisations, completions and zero-delay timeouts at `now` -- are dispatched
    // straight from the inbox without a round trip through the register queue.  Popping the
    // minimum of (queue U inbox) is exactly the full queue's order.
    int n_disp = 0;
    {
      double t = et;
      uint32_t k = ek;
      int p = target_proc(ep), pf = target_flow(ep);
      // queue head = entry 0 of set 0, held by lane 0
      const double head_t = pack_t((uint32_t)__builtin_amdgcn_readfirstlane((int)q.tlo[0]),
                                   (uint32_t)__builtin_amdgcn_readfirstlane((int)q.thi[0]));
      const uint32_t head_k = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.key[0]);
      for (;;) {
        S.h->now = t;
        S.h->cur_key = k;
        const unsigned long long td = prof ? __builtin_amdgcn_s_memtime() : 0;
        const int ptype = prof ? S.procs[p].type * 4 + (S.procs[p].state < 3 ? S.procs[p].state : 3) : 0;
        dispatch<BIG, TLDS>(S, K, T, p, pf);
        ++n_disp;
        if (prof && lane == 0) {
          a.prof_types[((long)env * 64 + ptype) * 2] += __builtin_amdgcn_s_memtime() - td;
          a.prof_types[((long)env * 64 + ptype) * 2 + 1] += 1;
        }
        const int ni = S.h->n_events;
        // pending-event high-water mark of the full queue (= host path's count after its last push)
        if (q.n + ni > S.h->max_events) S.h->max_events = q.n + ni;
        if (ni == 0 || n_disp >= 4096) break;
        int bi = 0;
        // (measured: keeping the last pushed event in registers to skip this LDS read when the
        // handler pushed exactly one event cost 44 VGPRs and was slower, 100.0k vs 104.0k env-steps/s)
        Event m = S.events[0];
        for (int i = 1; i < ni; ++i) {
          const Event c = S.events[i];
          if (ev_less(c, m)) { m = c; bi = i; }
        }
        if (!(m.t < head_t || (m.t == head_t && m.key < head_k))) break;
        remove_event(S, bi);
        t = m.t;
        k = m.key;
        p = m.proc;
        pf = m.flow;
      }
    }
    it += __builtin_amdgcn_readfirstlane(n_disp) - 1;
    // (measured: inserting a one-event inbox's event from registers instead of re-reading it here
    // was slower both with a second insert site, 97.3k vs 105.2k env-steps/s, and through the one
    // insert site, 101.3k vs 104.5k: the event kept live across the chain costs more than the read)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const unsigned long long t2 = prof ? __builtin_amdgcn_s_memtime() : 0;
    rq_merge_inbox<QS>(q, S, lane);
    if (prof) {
      const unsigned long long t3 = __builtin_amdgcn_s_memtime();
      t_sel += t1 - t0;
      t_hdl += t2 - t1;
      t_mrg += t3 - t2;
      n_ev += __builtin_amdgcn_readfirstlane(n_disp);
    }
  }
  const unsigned long long t_loop_end = prof ? __builtin_amdgcn_s_memtime() : 0;
  if (prof && lane == 0) {
    unsigned long long* pr = a.prof + (long)env * 4;
    pr[0] += t_sel;
    pr[1] += t_hdl;
    pr[2] += t_mrg;
    pr[3] += n_ev;
    a.prof_types[((long)env * 64 + 62) * 2] += t_begin - t_entry;  // prologue (topology stage, action, inbox)
    a.prof_types[((long)env * 64 + 62) * 2 + 1] += 1;
    a.prof_types[((long)env * 64 + 57) * 2] += t_act - t_entry;    // of which: topology stage + action load
    a.prof_types[((long)env * 64 + 57) * 2 + 1] += 1;
  }
  __syncthreads();
  // write the queue back (sorted) as the persistent pending-event array
  for (int s = 0; s < QS; ++s) {
    const int idx = s * 64 + lane;
    if (idx < q.n) {
      Event e;
      e.t = pack_t(q.tlo[s], q.thi[s]);
      e.key = q.key[s];
      e.proc = (int16_t)target_proc(q.proc[s]);
      e.flow = (int16_t)target_flow(q.proc[s]);
      S.events[idx] = e;
    }
  }
  if (lane == 0) S.h->n_events = q.n;
  __syncthreads();
  // epilogue: reward/stats in lane 0, observations lane-parallel (they read only LDS state)
  const long ostride = (long)K.n_pad * K.n_obs;
  int done = 0;
  if (lane == 0) {
    S.h->run_times++;
    finish_run_stats(S);
    const float r = compute_reward(S, K, T);
    write_stats(S, a.stats + (long)env * kNumStats);
    a.reward[env] = r;
    S.st->episode_return += r;
    S.h->run_count++;
    done = S.h->run_count >= K.episode_steps;
    a.done[env] = (uint8_t)done;
    if (done) a.ep_return[env] = (float)S.st->episode_return;
  }
  done = __builtin_amdgcn_readfirstlane(done);
  write_obs_wave(S, K, T.n, a.next_obs + env * ostride, done ? nullptr : a.obs + env * ostride, lane);
  if (done) {
    __syncthreads();
    {  // every lane (wave-uniform header copies), init loops spread over the lanes
      const int topo = a.topo_next[env];
      if (a.topo_cur && lane == 0) a.topo_cur[env] = topo;
      env_init<BIG>(S, K, a.topos[topo], topo, a.seeds[env], S.h->episode + 1, lane, 64);
    }
    __syncthreads();
    write_obs_wave(S, K, a.topos[a.topo_next[env]].n, a.obs + env * ostride, nullptr, lane);
  }
  if (lane == 0) *h_mem = h_reg;
  __syncthreads();
  if (PROF && lane == 0) {  // epilogue (queue write-back, reward, stats, observations, resets)
    a.prof_types[((long)env * 64 + 63) * 2] += __builtin_amdgcn_s_memtime() - t_loop_end;
    a.prof_types[((long)env * 64 + 63) * 2 + 1] += 1;
  }
}

// LDS_STATE: 0 = the state blob stays in HBM, 1 = the whole blob is staged in LDS, 2 = only its hot
// prefix is (the [N, C, S, N] schedule / WRR tables stay in HBM: 50- and 200-node topologies).
// TLDS: the topology tables are staged in LDS (SimContext: topo_stage_ > 0), known at compile time.
// GSC_SIM_MAX_SGPR (A/B builds only, scripts/sim_sgpr_ab.py): cap the step kernel's SGPR budget to measure what
// SGPR spills (to VGPR lanes) cost per spill
#ifdef GSC_SIM_MAX_SGPR
#define GSC_SIM_SGPR_ATTR __attribute__((amdgpu_num_sgpr(GSC_SIM_MAX_SGPR)))
#else
#define GSC_SIM_SGPR_ATTR
#endif
template <int QSETS, int LDS_STATE, bool PROF = false, bool TLDS = false>
__global__ __launch_bounds__(64) GSC_SIM_SGPR_ATTR void sim_step_kernel(SimArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  // The simulator step is the training loop's critical path (issue-bound, one wave per env) while
  // the learner runs concurrently with slack: give its waves issue priority over co-resident
  // learner waves on the same SIMD (GSC_SIM_PRIO, default 3; measured +0.6 %).
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  // LDS: [state blob or its hot prefix (LDS modes)][SimConst][topology tables]
  const long sbytes = a.lds_state_bytes;
  const long sb = LDS_STATE ? align16((int)sbytes) : 0;
  SimConst* Ks = reinterpret_cast<SimConst*>(smem + sb);
  if (lane == 0) *Ks = a.K;
  char* topo_lds = smem + sb + const_stage_bytes();
  char* g = a.states + (long)env * a.state_bytes;
  // diagnostic variant: shader-clock cycles and 100 MHz wall ticks over the whole workgroup (slots
  // 58 / 59) -> the effective engine clock while the simulator runs (e.g. beside the learner)
  const unsigned long long c_begin = PROF ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long r_begin = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
  if constexpr (LDS_STATE != 0) {
    const unsigned long long t0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
    copy16(smem, g, sbytes, lane);
    __syncthreads();
    const unsigned long long t1 = PROF ? __builtin_amdgcn_s_memtime() : 0;
    device_step_env<QSETS, PROF, LDS_STATE == 2, TLDS>(a, *Ks, smem, topo_lds, env, lane, LDS_STATE == 2 ? g : nullptr);
    const unsigned long long t2 = PROF ? __builtin_amdgcn_s_memtime() : 0;
    copy16(g, smem, sbytes, lane);
    if (PROF && lane == 0) {  // state blob HBM -> LDS / LDS -> HBM
      a.prof_types[((long)env * 64 + 60) * 2] += t1 - t0;
      a.prof_types[((long)env * 64 + 60) * 2 + 1] += 1;
      a.prof_types[((long)env * 64 + 61) * 2] += __builtin_amdgcn_s_memtime() - t2;
      a.prof_types[((long)env * 64 + 61) * 2 + 1] += 1;
    }
  } else {
    __syncthreads();
    device_step_env<QSETS, false, true, TLDS>(a, *Ks, g, topo_lds, env, lane);
  }
  if (PROF && lane == 0) {
    a.prof_types[((long)env * 64 + 58) * 2] += __builtin_amdgcn_s_memtime() - c_begin;
    a.prof_types[((long)env * 64 + 58) * 2 + 1] += 1;
    const unsigned long long r_end = __builtin_amdgcn_s_memrealtime();
    a.prof_types[((long)env * 64 + 59) * 2] += r_end - r_begin;
    // this step's wave start / end (100 MHz ticks; overwritten every step): dispatch skew vs wave duration
    a.prof_types[((long)env * 64 + 56) * 2] = r_begin;
    a.prof_types[((long)env * 64 + 56) * 2 + 1] = r_end;
    a.prof_types[((long)env * 64 + 59) * 2 + 1] += 1;
  }
}

// Positive-destination bitsets of every schedule row of this step's action block, for the placement walk of
// topologies beyond 64 nodes (controller_prologue<BIG>): one wave per (env, row) over the whole device,
// ahead of the step kernel (one HBM pass over the action block instead of a serial walk per env wave).
__global__ __launch_bounds__(256) void sim_pmask_kernel(SimArgs a) {
  const int env = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.y * 4 + (threadIdx.x >> 6);
  char* g = a.states + (long)env * a.state_bytes;
  const int n = a.topos[reinterpret_cast<const Header*>(g + a.L.hdr)->topo].n;  // topology of this step
  const int C = a.D.C, Sd = a.D.S;
  if (r >= n * C * Sd) return;
  const int sf = r % Sd, c = (r / Sd) % C, src = r / (Sd * C);
  if (sf >= a.K.F) return;  // not an action row (no chain position uses it)
  const float* row = a.actions + (long)env * a.action_stride + ((long)(src * a.K.C + c) * a.K.F + sf) * a.K.n_pad;
  uint64_t* pm = reinterpret_cast<uint64_t*>(g + a.L.pmask) + 4L * r;
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = 64 * q + lane < n ? row[64 * q + lane] : 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t b = (uint64_t)__ballot(v[q] > 0.f);
    if (lane == q) pm[q] = b;
  }
}

__global__ __launch_bounds__(64) void sim_reset_kernel(SimArgs a) {
  const int env = blockIdx.x;
  char* g = a.states + (long)env * a.state_bytes;
  if (threadIdx.x == 0) {
    Env S(g, a.L, a.D);
    reset_one(S, a, env);
  }
}

// ------------------------------------------------------------------------------------------------
// Host path (CPU tests, differential checks against the scalar oracle)
// ------------------------------------------------------------------------------------------------
static void host_step_env(const SimArgs& a, int env) {
  Env S(a.states + (long)env * a.state_bytes, a.L, a.D);
  const TopoDev& T = a.topos[S.h->topo];
  load_action(S, a.K, T, a.actions + (long)env * a.action_stride, 0, 1);
  controller_prologue(S, a.K, T);
  schedule_stop(S, a.K);
  run_until_stop_serial(S, a.K, T);
  step_epilogue(S, a, a.K, env);
}

template <class F>
static void parallel_for(int n, int threads, F&& fn) {
  threads = std::max(1, std::min(threads, n));
  if (threads == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (int i = t; i < n; i += threads) fn(i);
    });
  for (auto& th : pool) th.join();
}

// ------------------------------------------------------------------------------------------------
// Context object owned by Python
// ------------------------------------------------------------------------------------------------
#ifdef GSC_SIM_ISA_ONLY
// register / ISA analysis build (scripts/sim_resources.py): only the named instantiation
template __global__ void sim_step_kernel<GSC_SIM_ISA_ONLY>(SimArgs);
#else
// The instantiated step kernels: QS = register-queue sets (64 pending events each), LDS mode, cycle-counting
// variant, topology staged in LDS.  TLDS kernels exist for the whole-state-in-LDS mode (Abilene-class
// topologies, the headline); larger topologies read unstaged tables through generic pointers.
template <int QS>
static const void* step_kernel_q(int mode, bool prof, bool tlds) {
  if (mode == 1 && tlds) return prof ? (const void*)sim_step_kernel<QS, 1, true, true> : (const void*)sim_step_kernel<QS, 1, false, true>;
  if (mode == 1) return prof ? (const void*)sim_step_kernel<QS, 1, true, false> : (const void*)sim_step_kernel<QS, 1, false, false>;
  if (mode == 2) return prof ? (const void*)sim_step_kernel<QS, 2, true, false> : (const void*)sim_step_kernel<QS, 2, false, false>;
  if (mode == 0) return (const void*)sim_step_kernel<QS, 0, false, false>;  // (no cycle-counting variant)
  return nullptr;
}
static const void* step_kernel(int qs, int mode, bool prof, bool tlds) {
  switch (qs) {
    case 1: return step_kernel_q<1>(mode, prof, tlds);
    case 2: return step_kernel_q<2>(mode, prof, tlds);
    case 4: return step_kernel_q<4>(mode, prof, tlds);
    default: return step_kernel_q<8>(mode, prof, tlds);
  }
}

class SimContext {
 public:
  SimContext(py::dict dims, py::dict cfg, py::list topos, bool device, int host_threads)
      : device_(device), host_threads_(host_threads) {
    D_.N = dims["N"].cast<int>();
    D_.S = dims["S"].cast<int>();
    D_.C = dims["C"].cast<int>();
    D_.E = dims["E"].cast<int>();
    D_.flow_cap = dims["flow_cap"].cast<int>();
    D_.proc_cap = dims["proc_cap"].cast<int>();
    D_.event_cap = dims["event_cap"].cast<int>();
    D_.rel_cap = dims.contains("rel_cap") ? dims["rel_cap"].cast<int>() : D_.flow_cap;
    GSC_CHECK(D_.N <= 256, "at most 256 nodes per topology");
    GSC_CHECK(D_.flow_cap < 32768 && D_.proc_cap < 32768, "pool capacities must be < 32768");
    L_ = make_layout(D_);
    fill_const(cfg);
    for (auto item : topos) {
      py::dict t = item.cast<py::dict>();
      TopoDev td{};
      td.n = t["n"].cast<int>();
      td.E = t["E"].cast<int>();
      td.H = t["H"].cast<int>();
      td.n_ing = t["n_ing"].cast<int>();
      td.n_eg = t["n_eg"].cast<int>();
      td.diameter = t["diameter"].cast<double>();
      td.cap = ptr<const double>(t["cap"].cast<uintptr_t>());
      td.pdelay = ptr<const double>(t["pdelay"].cast<uintptr_t>());
      td.plen = ptr<const int16_t>(t["plen"].cast<uintptr_t>());
      td.pnodes = ptr<const int16_t>(t["pnodes"].cast<uintptr_t>());
      td.pedges = ptr<const int16_t>(t["pedges"].cast<uintptr_t>());
      td.phd = ptr<const double>(t["phd"].cast<uintptr_t>());
      td.edge_id = ptr<const int16_t>(t["edge_id"].cast<uintptr_t>());
      td.edge_cap = ptr<const double>(t["edge_cap"].cast<uintptr_t>());
      td.ingress = ptr<const int16_t>(t["ingress"].cast<uintptr_t>());
      td.egress = ptr<const int16_t>(t["egress"].cast<uintptr_t>());
      GSC_CHECK(td.n <= D_.N && td.E <= D_.E, "topology exceeds simulator dims");
      topos_.push_back(td);
    }
    GSC_CHECK(!topos_.empty(), "need at least one topology");
    if (device_) {
      GSC_HIP_CHECK(hipMalloc(&dev_topos_, sizeof(TopoDev) * topos_.size()));
      GSC_HIP_CHECK(hipMemcpy(dev_topos_, topos_.data(), sizeof(TopoDev) * topos_.size(), hipMemcpyHostToDevice));
      int dev = 0;
      GSC_HIP_CHECK(hipGetDevice(&dev));
      int max_lds = 0;
      GSC_HIP_CHECK(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
      int maxH = 1;
      for (auto& t : topos_) maxH = t.H > maxH ? t.H : maxH;
      topo_stage_ = topo_stage_bytes(D_, maxH);
      // Large topologies (N^2 * hops path tables beyond the LDS budget, e.g. 200 nodes): the tables
      // stay in HBM and are served from L2 — only SimConst (+ the state, if it fits) is staged.
      if (const_stage_bytes() + topo_stage_ + 1024 > max_lds) topo_stage_ = 0;
      // state in LDS: the whole blob, else its hot prefix (the schedule / WRR tables stay in HBM)
      const long total = L_.total, hot = L_.hot;
      auto fits = [&](long state) { return const_stage_bytes() + topo_stage_ + state <= max_lds; };
      auto fits_alone = [&](long state) { return const_stage_bytes() + state <= max_lds; };
      // the state has priority over the topology tables: every event reads and writes it, while the
      // tables are read-only and stay L2-resident (e.g. 50-node topologies: both do not fit one
      // workgroup's LDS together)
      if (topo_stage_ && !fits(total) && (fits_alone(total) || (!fits(hot) && fits_alone(hot)))) topo_stage_ = 0;
      lds_mode_ = fits(total) ? 1 : (fits(hot) ? 2 : 0);
      const long state = lds_mode_ == 1 ? total : (lds_mode_ == 2 ? hot : 0);
      const long fixed = const_stage_bytes() + topo_stage_;
      // the per-hop edge / delay tables save dependent lookups per hop, but not at the price of a workgroup
      // per CU below one wave per SIMD (50-node topologies with the state blob in HBM: 112 vs 72 KB of
      // tables).  Four env workgroups per CU (one per SIMD: the waves are issue-bound) are enough.
      if (topo_stage_) {
        const long without = topo_stage_bytes(D_, maxH, false);
        const long cu_lds = 160 * 1024;
        const long with_n = cu_lds / (const_stage_bytes() + topo_stage_ + state);
        if (with_n < 4 && with_n < cu_lds / (const_stage_bytes() + without + state)) {
          topo_stage_ = without;
          stage_pedges_ = 0;
        }
      }
      const long need = fixed + state;
      qsets_ = D_.event_cap <= 64 ? 1 : (D_.event_cap <= 128 ? 2 : (D_.event_cap <= 256 ? 4 : 8));
      if (need > 65536)
        for (int q : {1, 2, 4, 8})
          for (int m : {0, 1, 2})
            for (int pr : {0, 1})
              for (int tl : {0, 1})
                if (const void* f = step_kernel(q, m, pr, tl))
                  GSC_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need));
    }
  }
  ~SimContext() {
    if (dev_topos_) (void)hipFree(dev_topos_);
  }

  long state_bytes() const { return L_.total; }
  long hot_bytes() const { return L_.hot; }
  bool use_lds() const { return lds_mode_ != 0; }
  // 0: state in HBM, 1: whole state blob in LDS, 2: its hot prefix in LDS (schedule / WRR tables in HBM)
  int lds_mode() const { return lds_mode_; }
  bool uses_pmask() const { return device_ && lds_mode_ != 1 && pmask_rows(D_) > 0; }
  // where a producer of the action block may write the step kernel's destination bitsets (explore.hip PMask):
  // (offset of the pmask block in an env's state, its C and S dims), or None when the kernel does not read them
  py::object pmask_layout() const {
    if (!uses_pmask()) return py::none();
    return py::make_tuple((long)L_.pmask, D_.C, D_.S);
  }
  long lds_state() const { return lds_mode_ == 1 ? L_.total : (lds_mode_ == 2 ? L_.hot : 0); }
  // LDS bytes one env's workgroup needs on the device (SimConst + topology tables + staged state)
  long lds_per_env() const { return const_stage_bytes() + topo_stage_ + lds_state(); }

  void reset(uintptr_t states, uintptr_t topo_init, uintptr_t seeds, uintptr_t obs, int E, uintptr_t stream) {
    SimArgs a = args(states, topo_init, seeds, 0, 0, obs, 0, 0, 0, 0, 0, E);
    if (device_) {
      hipLaunchKernelGGL(sim_reset_kernel, dim3(E), dim3(64), 0, stream_of(stream), a);
      check_launch();
    } else {
      parallel_for(E, host_threads_, [&](int e) {
        Env S(a.states + (long)e * a.state_bytes, a.L, a.D);
        reset_one(S, a, e);
      });
    }
  }

  void step(uintptr_t states, uintptr_t topo_next, uintptr_t seeds, uintptr_t actions, long action_stride,
            uintptr_t obs, uintptr_t next_obs, uintptr_t reward, uintptr_t done, uintptr_t stats,
            uintptr_t ep_return, int E, uintptr_t stream, uintptr_t prof, uintptr_t topo_cur, bool pmask_ready) {
    SimArgs a = args(states, topo_next, seeds, actions, action_stride, obs, next_obs, reward, done, stats,
                     ep_return, E);
    a.topo_cur = ptr<int32_t>(topo_cur);
    a.prof = ptr<unsigned long long>(prof);
    a.prof_types = prof ? ptr<unsigned long long>(prof) + (long)E * 4 : nullptr;
    static const int prio = getenv("GSC_SIM_PRIO") ? atoi(getenv("GSC_SIM_PRIO")) : 3;
    a.prio = prio;
    if (device_) {
      const size_t lds = (size_t)lds_per_env();
      const hipStream_t st = stream_of(stream);
      // HBM-resident tables (BIG kernels), > 64 nodes; pmask_ready: the exploration kernel wrote the bitsets
      if (uses_pmask() && !pmask_ready) {
        hipLaunchKernelGGL(sim_pmask_kernel, dim3(E, (pmask_rows(D_) + 3) / 4), dim3(256), 0, st, a);
        check_launch();
      }
      // GSC_SIM_TLDS=0: the generic-pointer kernel even when the topology is staged (A/B diagnostics)
      static const bool tlds_ok = !(getenv("GSC_SIM_TLDS") && getenv("GSC_SIM_TLDS")[0] == '0');
      const bool tlds = tlds_ok && lds_mode_ == 1 && topo_stage_ > 0 && stage_pedges_;
      const void* f = step_kernel(qsets_, lds_mode_, a.prof != nullptr, tlds);
      GSC_CHECK(f, "no simulator kernel instantiated for this (queue sets, LDS mode, profiling) combination");
      hipLaunchKernelGGL(reinterpret_cast<void (*)(SimArgs)>(const_cast<void*>(f)), dim3(E), dim3(64), lds, st, a);
      check_launch();
    } else {
      parallel_for(E, host_threads_, [&](int e) { host_step_env(a, e); });
    }
  }

 private:
  SimArgs args(uintptr_t states, uintptr_t topo, uintptr_t seeds, uintptr_t actions, long action_stride,
               uintptr_t obs, uintptr_t next_obs, uintptr_t reward, uintptr_t done, uintptr_t stats,
               uintptr_t ep_return, int E) {
    SimArgs a{};
    a.states = ptr<char>(states);
    a.state_bytes = L_.total;
    a.lds_state_bytes = lds_state();
    a.L = L_;
    a.D = D_;
    a.K = K_;
    a.topos = device_ ? dev_topos_ : topos_.data();
    a.topo_next = ptr<const int32_t>(topo);
    a.seeds = ptr<const uint32_t>(seeds);
    a.actions = ptr<const float>(actions);
    a.action_stride = action_stride;
    a.obs = ptr<float>(obs);
    a.next_obs = ptr<float>(next_obs);
    a.reward = ptr<float>(reward);
    a.done = ptr<uint8_t>(done);
    a.stats = ptr<float>(stats);
    a.ep_return = ptr<float>(ep_return);
    a.E = E;
    a.use_lds = lds_mode_;
    a.topo_stage = topo_stage_;
    a.stage_pedges = stage_pedges_;
    return a;
  }

  void fill_const(py::dict c) {
    SimConst& K = K_;
    K = SimConst{};
    K.C = c["C"].cast<int>();
    K.S = c["S"].cast<int>();
    K.F = c["F"].cast<int>();
    GSC_CHECK(K.C <= kMaxC && K.S <= kMaxS && K.F <= kMaxF, "too many SFCs / SFs");
    GSC_CHECK(K.C == D_.C && K.S <= D_.S, "config/dims mismatch");  // D_.S may be padded (dims bucket)
    auto chain = c["chain"].cast<std::vector<std::vector<int>>>();
    GSC_CHECK((int)chain.size() == K.C, "chain list size");
    for (int i = 0; i < K.C; ++i) {
      GSC_CHECK((int)chain[i].size() <= K.F, "chain longer than F");
      K.chain_len[i] = (int)chain[i].size();
      for (size_t j = 0; j < chain[i].size(); ++j) {
        GSC_CHECK(chain[i][j] < K.F, "SF index must be < max chain length (reference action layout, Q19)");
        K.chain[i * kMaxF + j] = chain[i][j];
      }
    }
    auto pm = c["pd_mean"].cast<std::vector<double>>();
    auto ps = c["pd_std"].cast<std::vector<double>>();
    auto su = c["startup"].cast<std::vector<double>>();
    for (int s = 0; s < K.S; ++s) { K.pd_mean[s] = pm[s]; K.pd_std[s] = ps[s]; K.startup[s] = su[s]; }
    K.run_duration = c["run_duration"].cast<double>();
    K.det_arrival = c["det_arrival"].cast<int>();
    K.det_size = c["det_size"].cast<int>();
    K.dr_mean = c["dr_mean"].cast<double>();
    K.dr_std = c["dr_std"].cast<double>();
    K.size_shape = c["size_shape"].cast<double>();
    auto ttl = c["ttl"].cast<std::vector<double>>();
    GSC_CHECK(!ttl.empty() && (int)ttl.size() <= kMaxTTL, "ttl_choices size");
    K.n_ttl = (int)ttl.size();
    for (int i = 0; i < K.n_ttl; ++i) K.ttl[i] = ttl[i];
    K.inter_arr_mean = c["inter_arr_mean"].cast<double>();
    K.use_states = c["use_states"].cast<int>();
    K.mmpp_init = c["mmpp_init"].cast<int>();
    auto mm = c["mmpp_mean"].cast<std::vector<double>>();
    auto msw = c["mmpp_switch"].cast<std::vector<double>>();
    K.mmpp_mean[0] = mm[0]; K.mmpp_mean[1] = mm[1];
    K.mmpp_switch[0] = msw[0]; K.mmpp_switch[1] = msw[1];
    K.n_trace = c["n_trace"].cast<int>();
    K.trace_has_node = c["trace_has_node"].cast<int>();
    K.trace_time = ptr<const double>(c["trace_time"].cast<uintptr_t>());
    K.trace_node = ptr<const int16_t>(c["trace_node"].cast<uintptr_t>());
    K.trace_mean = ptr<const double>(c["trace_mean"].cast<uintptr_t>());
    K.trace_cap = ptr<const double>(c["trace_cap"].cast<uintptr_t>());
    auto feats = c["obs_feat"].cast<std::vector<int>>();
    K.n_obs = (int)feats.size();
    GSC_CHECK(K.n_obs >= 1 && K.n_obs <= 3, "1-3 observation features");
    for (int i = 0; i < K.n_obs; ++i) K.obs_feat[i] = feats[i];
    K.objective = c["objective"].cast<int>();
    K.w_flow = c["w_flow"].cast<double>();
    K.w_delay = c["w_delay"].cast<double>();
    K.w_node = c["w_node"].cast<double>();
    K.w_inst = c["w_inst"].cast<double>();
    K.target_success = c["target_success"].cast<double>();
    K.soft_deadline = c["soft_deadline"].cast<double>();
    K.dropoff = c["dropoff"].cast<double>();
    K.min_delay = c["min_delay"].cast<double>();
    K.diameter = c["diameter"].cast<double>();
    K.episode_steps = c["episode_steps"].cast<int>();
    K.n_pad = c["n_pad"].cast<int>();
    K.same_seed_every_episode = c["same_seed_every_episode"].cast<int>();
    GSC_CHECK(K.n_pad >= D_.N, "n_pad must be >= max nodes");
  }

  bool device_;
  int host_threads_;
  int lds_mode_ = 0;
  long topo_stage_ = 0;
  int stage_pedges_ = 1;
  int qsets_ = 8;
  Dims D_{};
  Layout L_{};
  SimConst K_{};
  std::vector<TopoDev> topos_;
  TopoDev* dev_topos_ = nullptr;
};

void register_sim(py::module_& m) {
  py::class_<SimContext>(m, "SimContext")
      .def(py::init<py::dict, py::dict, py::list, bool, int>(), py::arg("dims"), py::arg("cfg"), py::arg("topos"),
           py::arg("device"), py::arg("host_threads") = 8)
      .def_property_readonly("state_bytes", &SimContext::state_bytes)
      .def_property_readonly("use_lds", &SimContext::use_lds)
      .def_property_readonly("lds_per_env", &SimContext::lds_per_env)
      .def_property_readonly("lds_mode", &SimContext::lds_mode)
      .def_property_readonly("hot_bytes", &SimContext::hot_bytes)
      .def_property_readonly("pmask_layout", &SimContext::pmask_layout)
      .def("reset", &SimContext::reset)
      .def("step", &SimContext::step, py::arg("states"), py::arg("topo_next"), py::arg("seeds"), py::arg("actions"),
           py::arg("action_stride"), py::arg("obs"), py::arg("next_obs"), py::arg("reward"), py::arg("done"),
           py::arg("stats"), py::arg("ep_return"), py::arg("E"), py::arg("stream"), py::arg("prof") = 0,
           py::arg("topo_cur") = 0, py::arg("pmask_ready") = false);
  m.attr("SIM_NUM_STATS") = kNumStats;
  m.attr("SIM_HEADER_BYTES") = (int)sizeof(Header);
}
#endif  // GSC_SIM_ISA_ONLY

}  // namespace gsc
