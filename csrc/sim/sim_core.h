// Batched coord-sim core: one discrete-event environment per call, shared by the HIP kernel
// (one wave per env, state staged in LDS) and the host path (CPU tests / differential checks).
//
// Semantics follow the reference simulator (coordsim/, SimPy 4) and the scalar oracle in
// gsc_amd/coordsim/: every SimPy event id is reproduced (process initialise events are URGENT,
// timeouts and process completions NORMAL, FIFO on equal (time, priority)), so deterministic
// configurations agree bit-for-bit with the oracle.  Process instances are explicit state
// machines; see the per-process comments for the reference generator they implement.
#pragma once
#include "philox.h"

namespace gsc {

constexpr int kMaxC = 4;      // SFCs
constexpr int kMaxF = 8;      // chain length
constexpr int kMaxS = 8;      // distinct SFs
constexpr int kMaxTTL = 8;
constexpr int kNumStats = 16;

// (return_link_resources is no process here: a per-link release ledger, see ledger_push)
enum ProcType : uint8_t {
  P_FREE = 0, P_WRITER, P_MMPP, P_TRACE, P_ARRIVAL, P_HANDLE, P_DECIDE, P_FORWARD, P_PROCESS, P_REQUEST,
  P_FINISH
};
// per-type resume states
enum : uint8_t {
  W_BEGIN = 0, W_INIT, W_AFTER,
  M_START = 0, M_AFTER, M_UPDATE,
  TR_INIT = 0, TR_AFTER,
  A_LOOP = 0,
  H_LOOP = 0, H_AFTER_DECIDE, H_AFTER_FWD, H_AFTER_PROC,
  D_INIT = 0, D_RUN,
  F_INIT = 0, F_AFTER_HOP,
  PR_INIT = 0, PR_AFTER_REQ, PR_AFTER_WAIT,
  RQ_INIT = 0, RQ_AFTER,
  FI_INIT = 0, FI_AFTER
};
enum DropReason { R_TTL = 0, R_DECISION = 1, R_LINK = 2, R_NODE = 3 };
enum Objective { OBJ_PRIO_FLOW = 0, OBJ_SOFT_DEADLINE = 1, OBJ_SOFT_DEADLINE_EXP = 2, OBJ_WEIGHTED = 3 };
enum Flags {
  FLAG_FLOW_OVERFLOW = 1, FLAG_PROC_OVERFLOW = 2, FLAG_EVENT_OVERFLOW = 4, FLAG_BAD_STATE = 8, FLAG_REL_OVERFLOW = 16
};
constexpr int16_t kStopProc = -2;

struct alignas(16) Event {  // 16 B
  double t;
  uint32_t key;    // (priority << 31) | event id
  int16_t proc;
  int16_t flow;    // flow of the target process (-1: none): the dispatcher loads the process and its
                   // flow record concurrently instead of one after the other
};
// proc | flow << 16 (the register queue's 32-bit target word)
GSC_HD int32_t pack_target(int proc, int flow) {
  return (int32_t)((uint32_t)(uint16_t)proc | ((uint32_t)(uint16_t)flow << 16));
}
GSC_HD int target_proc(int32_t t) { return (int)(int16_t)(t & 0xffff); }
GSC_HD int target_flow(int32_t t) { return (int)(int16_t)((uint32_t)t >> 16); }

struct alignas(16) Proc {  // 32 B
  uint8_t type, state;
  int16_t flow, parent, a, b, c, ret, pad;
  double x;
  int16_t n1, e1, len, pad1;  // forwarder: the next hop's node / edge (prefetched), path length
};

// A pending link-capacity return: return_link_resources' timeout, keyed like the SimPy event it replaces.
struct alignas(8) Release {  // 24 B
  double t, dr;
  uint32_t key;
  int32_t edge;
};

struct alignas(16) Flow {  // 64 B = 16 dwords (one per lane in load_proc_flow)
  double dr, duration, e2e, ttl, creation;
  int32_t id;
  int16_t node, egress, sfc, pos, cur_sf, ingress;
  uint8_t departed, fwd_eg, dropped, proc_idx;
};

// Control state the event loop reads (device: held in registers for the whole window).
struct Header {
  double now;
  uint32_t eid;
  int32_t n_events, flow_top, proc_top;
  int32_t run_times, episode, run_count, topo;
  uint32_t key0, key1;
  uint64_t ctr;
  int32_t total_flow_count, trace_index, flags, n;
  int32_t max_events, max_procs, max_flows;
  int32_t proc_head;         // proc_free[proc_top - 1] (the next pid to allocate), cached off the LDS stack
  uint32_t cur_key;          // key of the event being dispatched (orders the release ledger against it)
  int32_t n_rel, max_rel;    // pending link releases, high-water mark
};

// Metric accumulators (reference coordsim/metrics/metrics.py): written by the handlers, read only by the
// epilogue (reward, stats).  Device: stay in LDS and are updated by one lane's LDS atomics (no read-back on
// the event loop's dependent chain, no registers held for them across the loop).
struct Stats {
  int32_t gen, processed, dropped, active;
  int32_t run_gen, run_processed, run_dropped, num_path_delays;
  int32_t drop_reason[4];
  int32_t num_proc_delays, pad0;
  double total_e2e, total_path_delay, total_proc_delay;
  double run_e2e, run_total_path_delay, run_avg_path_delay;
  uint64_t run_max_e2e;      // bits of a non-negative double (integer max == float max)
  double ewma_flows, episode_return;
};

// Read-only per-topology tables (device or host memory).
struct TopoDev {
  int n, E, H, n_ing, n_eg, pad;
  double diameter;
  const double* cap;        // [n]
  const double* pdelay;     // [n*n]
  const int16_t* plen;      // [n*n]
  const int16_t* pnodes;    // [n*n*H]
  const int16_t* pedges;    // [n*n*H] edge id of each path hop (from the previous path node)
  const double* phd;        // [n*n*H] delay of each path hop (pdelay[previous path node][hop])
  const int16_t* edge_id;   // [n*n]
  const double* edge_cap;   // [E]
  const int16_t* ingress;   // [n_ing]
  const int16_t* egress;    // [n_eg]
};

struct SimConst {
  int C, S, F;                       // sfcs, distinct SFs, action sf dim (max chain length)
  int chain_len[kMaxC];
  int chain[kMaxC * kMaxF];          // global SF index of each chain position
  double pd_mean[kMaxS], pd_std[kMaxS], startup[kMaxS];
  double run_duration;
  int det_arrival, det_size;
  double dr_mean, dr_std, size_shape;
  int n_ttl;
  double ttl[kMaxTTL];
  double inter_arr_mean;
  int use_states, mmpp_init;
  double mmpp_mean[2], mmpp_switch[2];
  int n_trace, trace_has_node;
  const double* trace_time;
  const int16_t* trace_node;         // -1: applies to every ingress
  const double* trace_mean;          // NaN = None
  const double* trace_cap;           // NaN = no cap column
  // observation / reward
  int n_obs;
  int obs_feat[3];                   // 0 ingress_traffic, 1 node_load, 2 node_cap
  int objective;
  double w_flow, w_delay, w_node, w_inst;
  double target_success;             // NaN = 'auto' (EWMA)
  double soft_deadline, dropoff, min_delay;
  double diameter;                   // <0: use topology APSP diameter
  int episode_steps;
  int n_pad;                         // model node padding (action/obs layout)
  int same_seed_every_episode;
};

struct Dims {
  int N, S, C, E, flow_cap, proc_cap, event_cap, rel_cap;
};

// The blob is [hot | cold]: everything the event handlers touch per event first, then the two
// [N, C, S, N] tables a WRR decision reads one row of (the schedule and the per-run flow counters).
// Topologies whose whole blob exceeds LDS (50 / 200 nodes: the tables alone are 270 KB / 4.3 MB)
// stage only the hot prefix [0, hot) in LDS and keep the cold tables in HBM (served from L2).
struct Layout {
  int hdr, stats, node_cap, node_rem, inter_arr, max_usage, run_drop_node, mmpp_state, sf_load, sf_start, proc_traffic,
      requested, drop_locs, link_rem, link_passed, link_next, rel, flows, procs, events, flow_free, proc_free,
      sf_present, placement, hot, sched, wrr, pmask, total;
};

// WRR counter rows ([N, C, S] rows of N counters) and the run-window epoch that tags them (see run_decide)
__host__ __device__ constexpr int wrr_rows(const Dims& d) { return d.N * d.C * d.S; }

// Topologies beyond one wave of destinations keep, per schedule row (src, c, sf), the bitset of its
// positive destinations (4 x 64 bits, n <= 256): the device placement walk ORs rows instead of
// re-reading them (see controller_prologue).  Absent (0 rows) for n <= 64.
__host__ __device__ constexpr int pmask_rows(const Dims& d) { return d.N > 64 ? d.N * d.C * d.S : 0; }

__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }
__host__ __device__ constexpr int wrr_ep_offset(const Layout& L, const Dims& d) {
  return L.hot - align16(4 * (wrr_rows(d) + 1));
}

__host__ __device__ constexpr Layout make_layout(const Dims& d) {
  Layout L{};
  int o = 0;
#define GSC_TAKE(field, bytes) L.field = o; o += align16((int)(bytes));
  GSC_TAKE(hdr, sizeof(Header));
  GSC_TAKE(stats, sizeof(Stats));
  GSC_TAKE(node_cap, 8 * d.N);
  GSC_TAKE(node_rem, 8 * d.N);
  GSC_TAKE(inter_arr, 8 * d.N);
  GSC_TAKE(max_usage, 8 * d.N);
  GSC_TAKE(run_drop_node, 4 * d.N);
  GSC_TAKE(mmpp_state, 4 * d.N);
  GSC_TAKE(sf_load, 8 * d.N * d.S);
  GSC_TAKE(sf_start, 8 * d.N * d.S);
  GSC_TAKE(proc_traffic, 8 * d.N * d.S);
  GSC_TAKE(requested, 8 * d.N * d.C * d.S);
  GSC_TAKE(drop_locs, 4 * d.N * (d.S + 1));
  GSC_TAKE(link_rem, 8 * d.E);
  GSC_TAKE(link_passed, 8 * d.E);
  GSC_TAKE(link_next, 8 * d.E);
  GSC_TAKE(rel, sizeof(Release) * d.rel_cap);
  GSC_TAKE(flows, sizeof(Flow) * d.flow_cap);
  GSC_TAKE(procs, sizeof(Proc) * d.proc_cap);
  GSC_TAKE(events, sizeof(Event) * d.event_cap);
  GSC_TAKE(flow_free, 2 * d.flow_cap);
  GSC_TAKE(proc_free, 2 * d.proc_cap);
  GSC_TAKE(sf_present, d.N * d.S);
  GSC_TAKE(placement, d.N * d.S);
  // the last run of the hot prefix: per-row WRR epoch + the current run-window epoch (wrr_ep_offset; not a
  // Layout field -- the kernel-argument layout of the LDS-resident kernels stays as it was)
  o += align16(4 * (wrr_rows(d) + 1));
  L.hot = o;
  GSC_TAKE(sched, 8 * d.N * d.C * d.S * d.N);
  GSC_TAKE(wrr, 4 * d.N * d.C * d.S * d.N);
  GSC_TAKE(pmask, 32 * pmask_rows(d));
#undef GSC_TAKE
  L.total = o;
  return L;
}

// Typed view of one env's state blob (the hot prefix at `base`, the cold tables at `cold`: the same
// blob unless the hot prefix was staged into LDS on its own).
struct Env {
  Header* h;
  Stats* st;
  double *node_cap, *node_rem, *inter_arr, *max_usage, *sf_load, *sf_start, *proc_traffic, *requested, *sched,
      *link_rem, *link_passed, *link_next;
  int32_t *run_drop_node, *mmpp_state, *drop_locs, *wrr;
  int32_t* wrr_ep;     // [wrr_rows + 1]: run-window epoch of each WRR counter row, then the current epoch
  const float* act;    // device kernels with HBM-resident schedule tables (BIG): this step's action block
                       // ([n_pad, C, F, n_pad] floats), read in place of the (double) schedule table
  uint64_t* pmask;
  Release* rel;
  Flow* flows;
  Proc* procs;
  Event* events;
  int16_t *flow_free, *proc_free;
  uint8_t *sf_present, *placement;
  Dims d;

  GSC_HD Env(char* base, const Layout& L, const Dims& dims, char* cold = nullptr) : d(dims) {
    char* const cb = cold ? cold : base;
    h = (Header*)(base + L.hdr);
    st = (Stats*)(base + L.stats);
    node_cap = (double*)(base + L.node_cap);
    node_rem = (double*)(base + L.node_rem);
    inter_arr = (double*)(base + L.inter_arr);
    max_usage = (double*)(base + L.max_usage);
    run_drop_node = (int32_t*)(base + L.run_drop_node);
    mmpp_state = (int32_t*)(base + L.mmpp_state);
    sf_load = (double*)(base + L.sf_load);
    sf_start = (double*)(base + L.sf_start);
    proc_traffic = (double*)(base + L.proc_traffic);
    requested = (double*)(base + L.requested);
    drop_locs = (int32_t*)(base + L.drop_locs);
    sched = (double*)(cb + L.sched);
    wrr = (int32_t*)(cb + L.wrr);
    wrr_ep = (int32_t*)(base + wrr_ep_offset(L, dims));
    act = nullptr;
    pmask = (uint64_t*)(cb + L.pmask);
    link_rem = (double*)(base + L.link_rem);
    link_passed = (double*)(base + L.link_passed);
    link_next = (double*)(base + L.link_next);
    rel = (Release*)(base + L.rel);
    flows = (Flow*)(base + L.flows);
    procs = (Proc*)(base + L.procs);
    events = (Event*)(base + L.events);
    flow_free = (int16_t*)(base + L.flow_free);
    proc_free = (int16_t*)(base + L.proc_free);
    sf_present = (uint8_t*)(base + L.sf_present);
    placement = (uint8_t*)(base + L.placement);
  }
};

// ------------------------------------------------------------------------------------------------
// RNG helpers (per-env Philox stream; deterministic configs draw nothing)
// ------------------------------------------------------------------------------------------------
// Random draws and the fp64 transcendental functions behind them are kept out of the event loop's
// instruction stream: on the device they are out-of-line functions taking scalars (the deterministic
// configurations, e.g. the headline's, never call them; inlined, Philox rounds and fp64 log / exp / cos
// sequences sat between the hot handler blocks -- ~30 % of the kernel's code).  Host: inline.
#if defined(__HIP_DEVICE_COMPILE__)
#define GSC_COLD __device__ __attribute__((noinline))
#else
#define GSC_COLD inline
#endif
GSC_COLD double rng_u01_draw(uint32_t k0, uint32_t k1, uint64_t c) {
  const Philox4 r = philox4x32_10(k0, k1, c);
  return u01_53(r.v[0], r.v[1]);
}
GSC_COLD double rng_normal_draw(uint32_t k0, uint32_t k1, uint64_t c, double mean, double std) {
  const Philox4 r = philox4x32_10(k0, k1, c);
  const double u1 = 1.0 - u01_53(r.v[0], r.v[1]);  // (0, 1]
  const double u2 = u01_53(r.v[2], r.v[3]);
  return mean + std * (sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}
GSC_COLD double exp_from_u01(double u, double mean) { return -log(1.0 - u) * mean; }     // expovariate(1/mean)
GSC_COLD double pareto_from_u01(double u, double shape) { return exp(-log(1.0 - u) / shape); }  // pareto + 1
GSC_COLD double log10_cold(double x) { return log10(x); }

GSC_HD uint32_t env_key(uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
#else
  return k;
#endif
}
GSC_HD double rng_u01(Env& S) { return rng_u01_draw(env_key(S.h->key0), env_key(S.h->key1), S.h->ctr++); }
GSC_HD double rng_normal(Env& S, double mean, double std) {
  if (std == 0.0) return mean;
  return rng_normal_draw(env_key(S.h->key0), env_key(S.h->key1), S.h->ctr++, mean, std);
}
GSC_HD int rng_int(Env& S, int n) {
  if (n <= 1) return 0;
  int k = (int)(rng_u01(S) * n);
  return k >= n ? n - 1 : k;
}

// ------------------------------------------------------------------------------------------------
// Wave-parallel helpers (device): the handlers run wave-uniform (every lane holds the same state),
// so a loop over nodes / destinations can spread over the 64 lanes and reduce with DPP.
// ------------------------------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ int wave_lane() { return (int)__lane_id(); }
// DPP row_shr:1,2,4,8 + row_bcast:15,31: lane 63 ends up with the reduction of all 64 lanes
template <class OP>
__device__ __forceinline__ uint32_t dpp_red_u32(uint32_t v, uint32_t ident, OP op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x111, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x112, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x114, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x118, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x142, 0xA, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ int wave_sum_i32(int v) {
  return (int)dpp_red_u32((uint32_t)v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// max of a double over the wave (exact), broadcast to every lane
__device__ __forceinline__ double wave_max_f64(double v) {
  const int ilo = 0, ihi = (int)0xFFF00000u;  // -inf
#define GSC_DPP_MAXD(ctrl, rm)                                                                  \
  {                                                                                            \
    const int lo = __builtin_amdgcn_update_dpp(ilo, __double2loint(v), ctrl, rm, 0xF, false);  \
    const int hi = __builtin_amdgcn_update_dpp(ihi, __double2hiint(v), ctrl, rm, 0xF, false);  \
    const double o = __hiloint2double(hi, lo);                                                 \
    v = o > v ? o : v;                                                                         \
  }
  GSC_DPP_MAXD(0x111, 0xF) GSC_DPP_MAXD(0x112, 0xF) GSC_DPP_MAXD(0x114, 0xF) GSC_DPP_MAXD(0x118, 0xF)
  GSC_DPP_MAXD(0x142, 0xA) GSC_DPP_MAXD(0x143, 0xC)
#undef GSC_DPP_MAXD
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                          __builtin_amdgcn_readlane(__double2loint(v), 63));
}
#endif

// Topology-table read.  TLDS (device kernels whose topology tables are staged in LDS, known at compile
// time): the generic table pointer is cast to the LDS address space, so the read is a ds_read rather
// than a flat load (which waits on both the vector-memory and the LDS counters).
template <bool TLDS, class V>
GSC_HD V tab(const V* p, long i) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (TLDS) return ((const __attribute__((address_space(3))) V*)p)[i];
#endif
  return p[i];
}

// ------------------------------------------------------------------------------------------------
// Event / process primitives (SimPy contract)
// ------------------------------------------------------------------------------------------------
GSC_HD void push_event(Env& S, double t, uint32_t prio, int16_t proc, int16_t flow) {
  Header* h = S.h;
  const uint32_t key = (prio << 31) | (h->eid & 0x7fffffffu);
  h->eid++;
  if (h->n_events >= S.d.event_cap) { h->flags |= FLAG_EVENT_OVERFLOW; return; }
  Event e;
  e.t = t;
  e.key = key;
  e.proc = proc;
  e.flow = flow;
  S.events[h->n_events++] = e;
  if (h->n_events > h->max_events) h->max_events = h->n_events;
}
// yield env.timeout(delay) of process pid (whose flow is `flow`)
GSC_HD void timeout(Env& S, int pid, int flow, double delay) {
  push_event(S, S.h->now + delay, 1u, (int16_t)pid, (int16_t)flow);
}

GSC_HD int alloc_proc(Env& S, uint8_t type, uint8_t state, int flow, int parent) {
  Header* h = S.h;
  if (h->proc_top <= 0) { h->flags |= FLAG_PROC_OVERFLOW; return -1; }
  // the stack top is cached in the header: no dependent LDS read before the new record is written;
  // the next top is loaded now and only needed by the next allocation
  const int pid = GSC_UNI(h->proc_head);
  --h->proc_top;
  h->proc_head = h->proc_top > 0 ? (int)S.proc_free[h->proc_top - 1] : -1;
  Proc& p = S.procs[pid];
  p.type = type; p.state = state; p.flow = (int16_t)flow; p.parent = (int16_t)parent;
  p.a = p.b = p.c = p.ret = 0; p.x = 0.0;
  p.n1 = p.e1 = p.len = p.pad1 = 0;
  const int used = S.d.proc_cap - h->proc_top;
  if (used > h->max_procs) h->max_procs = used;
  return pid;
}
// env.process(gen): new process + URGENT initialise event.
GSC_HD int spawn(Env& S, uint8_t type, uint8_t state, int flow, int parent) {
  const int pid = alloc_proc(S, type, state, flow, parent);
  if (pid < 0) { S.h->eid++; return -1; }
  push_event(S, S.h->now, 0u, (int16_t)pid, (int16_t)flow);
  return pid;
}
// A process yields env.process(itself-again): re-initialise the same slot (recursive reference generators).
GSC_HD void respawn_self(Env& S, int pid, uint8_t state) {  // writer / MMPP / trace processes (no flow)
  S.procs[pid].state = state;
  push_event(S, S.h->now, 0u, (int16_t)pid, (int16_t)-1);
}
// Generator return: completion event (NORMAL, delay 0); resumes the waiting parent if any.
// P = the returning process's record (a parent always serves the same flow as its child).
GSC_HD void proc_return(Env& S, int pid, const Proc& P, int16_t value) {
  const int parent = GSC_UNI(P.parent);
  if (parent >= 0) {
    S.procs[parent].ret = value;
    push_event(S, S.h->now, 1u, (int16_t)parent, P.flow);
  } else {
    S.h->eid++;
  }
  S.procs[pid].type = P_FREE;
  S.proc_free[S.h->proc_top++] = (int16_t)pid;
  S.h->proc_head = pid;
}

GSC_HD int alloc_flow(Env& S) {
  Header* h = S.h;
  if (h->flow_top <= 0) { h->flags |= FLAG_FLOW_OVERFLOW; return -1; }
  const int fid = GSC_UNI(S.flow_free[--h->flow_top]);
  const int used = S.d.flow_cap - h->flow_top;
  if (used > h->max_flows) h->max_flows = used;
  return fid;
}
GSC_HD void free_flow(Env& S, int fid) { S.flow_free[S.h->flow_top++] = (int16_t)fid; }

// ------------------------------------------------------------------------------------------------
// Link-capacity returns as a per-link ledger (DefaultFlowForwarder.return_link_resources,
// default_forwarder.py:112-125: after each hop a process waits flow.duration, then adds flow.dr back
// to the link).  The forwarder's hop step spawns that process and yields; the next event is always
// its URGENT initialise event (no other URGENT event can be pending at the time of a NORMAL hop
// timeout), whose only action is the duration timeout.  So the return takes effect exactly at
// (now + duration, NORMAL, the event id drawn right after the forwarder's own event), and its
// completion event has no waiter.  The ledger records that key instead of the three SimPy events;
// a capacity check of link e at event (t, key) first applies e's entries with a smaller key, in key
// order.  Event ids of the replaced events are not drawn: every remaining event and ledger key keeps
// its relative order, so the outcome is bit-identical (tests/test_batched_sim_diff.py) with about a
// quarter fewer dispatched events per step.
// ------------------------------------------------------------------------------------------------
GSC_HD bool key_less(double ta, uint32_t ka, double tb, uint32_t kb) { return ta < tb || (ta == tb && ka < kb); }

GSC_HD void ledger_push(Env& S, double t, int e, double dr) {
  Header* h = S.h;
  const uint32_t key = (1u << 31) | (h->eid & 0x7fffffffu);
  h->eid++;
  if (h->n_rel >= S.d.rel_cap) { h->flags |= FLAG_REL_OVERFLOW; return; }
  Release r;
  r.t = t;
  r.dr = dr;
  r.key = key;
  r.edge = e;
  S.rel[h->n_rel++] = r;
  if (h->n_rel > h->max_rel) h->max_rel = h->n_rel;
  if (t < S.link_next[e]) S.link_next[e] = t;
}

// Apply link e's returns that precede the current event, in key order, then refresh link_next[e].
GSC_HD_CALL void ledger_apply(Env& S, int e, double lnext) {
  const double now = S.h->now;
  if (GSC_UNI(now < lnext)) return;  // nothing due (the common case)
  const uint32_t ck = S.h->cur_key;
#if defined(__HIP_DEVICE_COMPILE__)
  const int lane = wave_lane();
  {
    // fast path (at most 64 pending returns, exactly one of them due): one entry per lane, the due
    // one found by a ballot, link_next from the same pass
    const int nr = GSC_UNI(S.h->n_rel);
    if (nr <= 64) {
      Release r;
      r.t = 1.0 / 0.0;
      r.dr = 0.0;
      r.edge = -1;
      r.key = 0xffffffffu;
      if (lane < nr) r = S.rel[lane];
      const bool mine = r.edge == e;
      const unsigned long long due = __ballot(mine && key_less(r.t, r.key, now, ck));
      if (due == 0) return;  // returns of link e at this time with a later key: nothing to apply
      if (__popcll(due) == 1) {
        const int idx = (int)__ffsll((long long)due) - 1;
        S.link_rem[e] += readlane_f64(r.dr, idx);
        // link_next = the earliest remaining return of link e: usually none or one (no wave reduction)
        const unsigned long long rest = __ballot(mine && lane != idx);
        const int nrest = __popcll(rest);
        S.link_next[e] = nrest == 0 ? 1.0 / 0.0
                         : nrest == 1 ? readlane_f64(r.t, (int)__ffsll((long long)rest) - 1)
                                      : -wave_max_f64(-(mine && lane != idx ? r.t : 1.0 / 0.0));
        const int last = nr - 1;
        if (idx != last) S.rel[idx] = S.rel[last];
        S.h->n_rel = last;
        __builtin_amdgcn_wave_barrier();
        return;
      }
    }
  }
  for (;;) {  // general case: repeatedly the smallest due entry (wave min over (t, key))
    const int nr = GSC_UNI(S.h->n_rel);
    double bt = 1.0 / 0.0;
    uint32_t bk = 0xffffffffu;
    int bi = -1;
    for (int i = lane; i < nr; i += 64) {
      const Release r = S.rel[i];
      if (r.edge == e && key_less(r.t, r.key, now, ck) && key_less(r.t, r.key, bt, bk)) { bt = r.t; bk = r.key; bi = i; }
    }
    const double tmin = -wave_max_f64(-bt);
    const uint32_t kmin = dpp_red_u32(bt == tmin ? bk : 0xffffffffu, 0xffffffffu,
                                      [](uint32_t a, uint32_t b) { return a < b ? a : b; });
    if (kmin == 0xffffffffu) break;
    const unsigned long long who = __ballot(bi >= 0 && bt == tmin && bk == kmin);
    const int idx = __builtin_amdgcn_readlane(bi, (int)__ffsll((long long)who) - 1);
    S.link_rem[e] += S.rel[idx].dr;
    const int last = nr - 1;
    if (idx != last) S.rel[idx] = S.rel[last];
    S.h->n_rel = last;
    __builtin_amdgcn_wave_barrier();
  }
  double nx = 1.0 / 0.0;
  for (int i = lane; i < S.h->n_rel; i += 64) {
    const Release r = S.rel[i];
    if (r.edge == e && r.t < nx) nx = r.t;
  }
  S.link_next[e] = -wave_max_f64(-nx);
#else
  for (;;) {
    int bi = -1;
    for (int i = 0; i < S.h->n_rel; ++i) {
      const Release& r = S.rel[i];
      if (r.edge == e && key_less(r.t, r.key, now, ck) &&
          (bi < 0 || key_less(r.t, r.key, S.rel[bi].t, S.rel[bi].key)))
        bi = i;
    }
    if (bi < 0) break;
    S.link_rem[e] += S.rel[bi].dr;
    const int last = --S.h->n_rel;
    if (bi != last) S.rel[bi] = S.rel[last];
  }
  double nx = 1.0 / 0.0;
  for (int i = 0; i < S.h->n_rel; ++i)
    if (S.rel[i].edge == e && S.rel[i].t < nx) nx = S.rel[i].t;
  S.link_next[e] = nx;
#endif
}

// ------------------------------------------------------------------------------------------------
// Metrics hooks (reference coordsim/metrics/metrics.py)
// ------------------------------------------------------------------------------------------------
// Make lane-parallel LDS writes of this wave visible to the (uniform) reads that follow.
GSC_HD void lanes_sync(int ls) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (ls > 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
#else
  (void)ls;
#endif
}

// l0 / ls: this lane and the lane count sharing the work (device: wave_lane(), 64; host or a
// single active lane: 0, 1)
// BIG (device kernels whose [N, C, S, N] tables stay in HBM): the WRR counters are not zeroed here --
// the run-window epoch advances and a decision zeroes a counter row the first time the window uses it
// (200 nodes: 1.4 MB of counters per env and window otherwise, written by one wave)
template <bool BIG = false>
GSC_HD_CALL void reset_run_metrics(Env& S, const SimConst& K, int n, int l0, int ls) {
  Stats* st = S.st;
  st->run_gen = st->run_processed = st->run_dropped = 0;
  st->run_e2e = st->run_total_path_delay = st->run_avg_path_delay = 0.0;
  st->run_max_e2e = 0;
  const int N = S.d.N, Sd = S.d.S, C = S.d.C;
  for (int v = l0; v < N; v += ls) { S.run_drop_node[v] = 0; S.max_usage[v] = 0.0; }
  for (int i = l0; i < N * Sd; i += ls) S.proc_traffic[i] = 0.0;
  for (int i = l0; i < N * C * Sd; i += ls) S.requested[i] = 0.0;
  if constexpr (BIG) {
    const int ep = S.wrr_ep[wrr_rows(S.d)] + 1;  // every lane reads, then writes, the same value
    lanes_sync(ls);
    S.wrr_ep[wrr_rows(S.d)] = ep;
  } else {
    for (int i = l0; i < N * C * Sd * N; i += ls) S.wrr[i] = 0;
  }
  lanes_sync(ls);
  (void)K; (void)n;
}

// Device: one lane updates the accumulators with LDS atomics (every lane runs the handler; the others
// skip), in program order -- the same sums, in the same order, as the host's plain updates.
#if defined(__HIP_DEVICE_COMPILE__)
#define GSC_ST_LANE0 if (wave_lane() == 0)
template <class T, class V>
__device__ __forceinline__ void st_add(T* p, V v) {
  __hip_atomic_fetch_add(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_max(uint64_t* p, uint64_t v) {
  __hip_atomic_fetch_max((unsigned long long*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#else
#define GSC_ST_LANE0
template <class T, class V>
inline void st_add(T* p, V v) { *p += (T)v; }
inline void st_max(uint64_t* p, uint64_t v) { if (v > *p) *p = v; }
#endif
GSC_HD uint64_t dbits(double x) {
  uint64_t u;
  __builtin_memcpy(&u, &x, 8);
  return u;
}

GSC_HD_CALL void dropped_flow(Env& S, const Flow& f, int reason) {
  const int sf = GSC_UNI(f.cur_sf < 0 ? S.d.S : f.cur_sf), node = GSC_UNI(f.node);
  if (GSC_UNI(f.ttl <= 0)) reason = R_TTL;
  Stats* st = S.st;
  GSC_ST_LANE0 {
    st_add(&st->dropped, 1);
    st_add(&st->active, -1);
    st_add(&st->run_dropped, 1);
    st_add(&S.drop_locs[node * (S.d.S + 1) + sf], 1);
    st_add(&S.run_drop_node[node], 1);
    st_add(&st->drop_reason[reason], 1);
  }
}

GSC_HD_CALL void completed_flow(Env& S, const Flow& f) {
  Stats* st = S.st;
  GSC_ST_LANE0 {
    st_add(&st->processed, 1);
    st_add(&st->run_processed, 1);
    st_add(&st->active, -1);
    st_add(&st->total_e2e, f.e2e);
    st_add(&st->run_e2e, f.e2e);
    st_max(&st->run_max_e2e, dbits(f.e2e));  // e2e >= 0
  }
}

// (run_avg_path_delay = run_total_path_delay / run_gen is derived in the epilogue: nothing reads it
// inside the window)
GSC_HD void add_path_delay(Env& S, double d) {
  Stats* st = S.st;
  GSC_ST_LANE0 {
    st_add(&st->num_path_delays, 1);
    st_add(&st->total_path_delay, d);
    st_add(&st->run_total_path_delay, d);
  }
}

// ------------------------------------------------------------------------------------------------
// Process handlers
//
// Each handler works on register copies of its process record (and flow record) — two/four
// 16-byte LDS loads — and writes back only what it changed before yielding.  A process that
// returns is freed by proc_return (its record is never written back afterwards).
// ------------------------------------------------------------------------------------------------
GSC_HD void end_flow(Env& S, int pid, const Proc& P, int fid) {
  free_flow(S, fid);
  proc_return(S, pid, P, 0);
}

// FlowSimulator.handle_flow (flowsimulator.py:72-128)
// Handlers receive the dispatched process record P and (for flow processes) the flow record f,
// both loaded by dispatch() concurrently; they write back only what they change.
GSC_HD_CALL void run_handle(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P, const Flow& f) {
  const int fid = GSC_UNI(P.flow);
  int state = GSC_UNI(P.state);
  for (;;) {
    switch (state) {
      case H_LOOP:
        if (GSC_UNI(f.departed)) {
          completed_flow(S, f);
          end_flow(S, pid, P, fid);
          return;
        }
        S.procs[pid].state = H_AFTER_DECIDE;
        spawn(S, P_DECIDE, D_INIT, fid, pid);
        return;
      case H_AFTER_DECIDE: {
        const int nxt = GSC_UNI(P.ret);
        if (nxt < 0) { dropped_flow(S, f, R_DECISION); end_flow(S, pid, P, fid); return; }
        S.procs[pid].state = H_AFTER_FWD;
        const int c = spawn(S, P_FORWARD, F_INIT, fid, pid);
        if (c >= 0) S.procs[c].b = (int16_t)nxt;
        return;
      }
      case H_AFTER_FWD:
        if (!GSC_UNI(P.ret)) { dropped_flow(S, f, R_LINK); end_flow(S, pid, P, fid); return; }
        if (!GSC_UNI(f.fwd_eg)) {
          S.procs[pid].state = H_AFTER_PROC;
          spawn(S, P_PROCESS, PR_INIT, fid, pid);
          return;
        }
        state = H_LOOP;
        break;
      case H_AFTER_PROC:
        if (!GSC_UNI(P.ret)) { dropped_flow(S, f, R_NODE); end_flow(S, pid, P, fid); return; }
        state = H_LOOP;
        break;
      default:
        S.h->flags |= FLAG_BAD_STATE;
        return;
    }
  }
  (void)K; (void)T;
}

// DefaultDecisionMaker.decide_next_node (default_decision_maker.py:18-81): weighted round robin.
// BIG (device kernels whose state is not LDS-resident: 50 / 200 nodes): counters + weights are loaded
// in one round trip (the rows are in HBM); the LDS-resident kernels compile the original two-pass scan
// (their register allocation is sensitive to any change).
template <bool BIG = false>
GSC_HD_CALL void run_decide(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P, const Flow& f) {
  if (GSC_UNI(P.state) == D_INIT) {
    S.procs[pid].state = D_RUN;
    timeout(S, pid, P.flow, 0.0);
    return;
  }
  const int fid = GSC_UNI(P.flow);
  if (GSC_UNI(f.ttl <= 0)) { proc_return(S, pid, P, -1); return; }
  if (GSC_UNI(f.fwd_eg)) {
    const int eg = GSC_UNI(f.egress), node = GSC_UNI(f.node);
    if (eg < 0) S.flows[fid].egress = (int16_t)node;
    proc_return(S, pid, P, (int16_t)(eg < 0 ? node : eg));
    return;
  }
  const int N = S.d.N, Sd = S.d.S, C = S.d.C, n = GSC_UNI(T.n);
  const int node = GSC_UNI(f.node), sfc = GSC_UNI(f.sfc);
  const int sf = GSC_UNI(K.chain[sfc * kMaxF + GSC_UNI(f.pos)]);
  S.flows[fid].cur_sf = (int16_t)sf;
  S.requested[(node * C + sfc) * Sd + sf] += f.dr;
  const int rid = (node * C + sfc) * Sd + sf;
  const int row = rid * N;
  const double* p = S.sched + row;
  int32_t* cnt = S.wrr + row;
#if defined(__HIP_DEVICE_COMPILE__)
  // destinations over the lanes: total by a DPP sum, the first destination with the largest
  // (weight - served ratio) by a DPP max + ballot (== the serial strict-greater scan)
  const int lane = wave_lane();
  double lbest = -1e300;
  int lidx = 0x7fffffff;
  if constexpr (BIG) {
    // weights straight from this step's action block (float -> double is exact: the same values as the
    // host path's double schedule table); counters of a row not yet used in this run window are stale
    // (zero): the row is zeroed now and tagged with the window's epoch (reset_run_metrics<BIG>)
    const float* pa = S.act + ((long)(node * K.C + sfc) * K.F + sf) * K.n_pad;
    const int ep = S.wrr_ep[wrr_rows(S.d)];
    const bool stale = GSC_UNI(S.wrr_ep[rid] != ep);
    int c4[4];  // n <= 256 (SimContext checks N <= 256): four destinations per lane
    double p4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = lane + 64 * j;
      const bool in = d < n;
      c4[j] = in ? cnt[d] : 0;
      p4[j] = in ? (double)pa[d] : 0.0;
    }
    if (stale) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c4[j] = 0;
        if (lane + 64 * j < n) cnt[lane + 64 * j] = 0;
      }
    }
    const int total = wave_sum_i32(c4[0] + c4[1] + c4[2] + c4[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = lane + 64 * j;
      const double ratio = total > 0 ? (double)c4[j] / (double)total : 0.0;
      const double diff = p4[j] > 0 ? p4[j] - ratio : -1.0;
      if (d < n && diff > lbest) { lbest = diff; lidx = d; }
    }
    const double best_v = wave_max_f64(lbest);
    const uint32_t cand = lbest == best_v ? (uint32_t)lidx : 0x7fffffffu;
    const int best = GSC_UNI((int)dpp_red_u32(cand, 0x7fffffffu, [](uint32_t a, uint32_t b) { return a < b ? a : b; }));
    // the chosen counter from the lane that loaded it (no re-read after the zeroing stores)
    int cb = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lane + 64 * j == best) cb = c4[j];
    const int old = GSC_UNI(__builtin_amdgcn_readlane(cb, best & 63));
    __builtin_amdgcn_wave_barrier();
    cnt[best] = old + 1;
    if (stale) S.wrr_ep[rid] = ep;
    proc_return(S, pid, P, (int16_t)best);
    return;
  } else {
    int part = 0;
    for (int d = lane; d < n; d += 64) part += cnt[d];
    const int total = wave_sum_i32(part);
    for (int d = lane; d < n; d += 64) {
      const double ratio = total > 0 ? (double)cnt[d] / (double)total : 0.0;
      const double diff = p[d] > 0 ? p[d] - ratio : -1.0;
      if (diff > lbest) { lbest = diff; lidx = d; }
    }
  }
  const double best_v = wave_max_f64(lbest);
  // lanes holding the max: the smallest destination index among them
  const uint32_t cand = lbest == best_v ? (uint32_t)lidx : 0x7fffffffu;
  int best = (int)dpp_red_u32(cand, 0x7fffffffu, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
  best = GSC_UNI(best);
#else
  int total = 0;
  for (int d = 0; d < n; ++d) total += cnt[d];
  int best = 0;
  double best_v = -1e300;
  for (int d = 0; d < n; ++d) {
    const double ratio = total > 0 ? (double)cnt[d] / (double)total : 0.0;
    const double diff = p[d] > 0 ? p[d] - ratio : -1.0;
    if (diff > best_v) { best_v = diff; best = d; }
  }
#endif
  cnt[best]++;
  proc_return(S, pid, P, (int16_t)best);
}

// DefaultFlowForwarder.forward_flow (default_forwarder.py:21-90); return_link_resources -> ledger_push.
// The record carries the path state: a = path source, b = destination, c = index of the hop just
// scheduled, ret / pad = its node / edge (its capacity return is recorded after the hop's timeout),
// x = path delay, len = path length, n1 / e1 = the NEXT hop's node / edge, prefetched when this hop was
// scheduled.  So a hop event needs one LDS round trip after the dispatch load: the link's capacity, next
// return time and passed-traffic counter, read together with the following hop's node / edge / delay.
template <bool BIG = false, bool TLDS = false>
GSC_HD_CALL void run_forward(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P0, const Flow& f0) {
  Proc P = P0;
  const int fid = GSC_UNI(P.flow);
  Flow f = f0;
  const int n = GSC_UNI(T.n), H = GSC_UNI(T.H);
  const int nxt = GSC_UNI(P.b);
  int rel_e = -1;  // link of the hop just taken: its capacity return is recorded after this step's event
  int c, hop, e;   // the hop to take now: index on the path, node, edge
  long pidx;
  if (GSC_UNI(P.state) == F_INIT) {
    const int cur = GSC_UNI(f.node);
    const int row = cur * n + nxt;
    pidx = (long)row * H;
    // path delay, length and the first two hops in one round trip (H > 1: pidx + 1 stays in the table)
    const double pd = (cur != nxt) ? tab<TLDS>(T.pdelay, row) : 0.0;
    const int len = tab<TLDS>(T.plen, row);
    hop = tab<TLDS>(T.pnodes, pidx);
    e = tab<TLDS>(T.pedges, pidx);
    P.n1 = H > 1 ? tab<TLDS>(T.pnodes, pidx + 1) : (int16_t)-1;
    P.e1 = H > 1 ? tab<TLDS>(T.pedges, pidx + 1) : (int16_t)-1;
    if (GSC_UNI(f.ttl - pd <= 0)) { S.flows[fid].ttl = 0; proc_return(S, pid, P, 0); return; }
    if (GSC_UNI(cur == f.egress && f.fwd_eg)) { f.departed = 1; S.flows[fid].departed = 1; }
    if (cur == nxt) { proc_return(S, pid, P, 1); return; }
    P.a = (int16_t)cur;
    P.len = (int16_t)len;
    P.x = pd;
    c = 0;
    hop = GSC_UNI(hop);
    e = GSC_UNI(e);
  } else {  // F_AFTER_HOP
    const int pc = GSC_UNI(P.c);
    rel_e = GSC_UNI(P.pad);
    f.node = (int16_t)GSC_UNI(P.ret);
    c = pc + 1;
    if (GSC_UNI(c >= P.len)) {
      add_path_delay(S, P.x);
      f.e2e += P.x;
      f.ttl -= P.x;
      Flow& fm = S.flows[fid];
      fm.node = f.node;
      fm.e2e = f.e2e;
      fm.ttl = f.ttl;
      proc_return(S, pid, P, 1);
      ledger_push(S, S.h->now + f.duration, rel_e, f.dr);
      return;
    }
    pidx = (long)(GSC_UNI(P.a) * n + nxt) * H + c;
    hop = GSC_UNI(P.n1);
    e = GSC_UNI(P.e1);
    // the hop after this one (c + 1 < H: still inside this path's row)
    P.n1 = c + 1 < H ? tab<TLDS>(T.pnodes, pidx + 1) : (int16_t)-1;
    P.e1 = c + 1 < H ? tab<TLDS>(T.pedges, pidx + 1) : (int16_t)-1;
  }
  // this hop's link state and delay, loaded together (the ledger check needs no separate round trip)
  const double lnext = S.link_next[e];
  double lrem = S.link_rem[e];
  const double lpass = S.link_passed[e];
  const double hd = tab<TLDS>(T.phd, pidx);  // == pdelay[previous path node][hop]
  Flow& fm = S.flows[fid];
  fm.node = f.node;
  if (GSC_UNI(!(S.h->now < lnext))) {  // capacity returns of this link are due first
    ledger_apply(S, e, lnext);
    lrem = S.link_rem[e];
  }
  if (GSC_UNI(lrem - f.dr >= 0)) {
    S.link_rem[e] = lrem - f.dr;
  } else {
    proc_return(S, pid, P, 0);
    if (rel_e >= 0) ledger_push(S, S.h->now + f.duration, rel_e, f.dr);
    return;
  }
  S.link_passed[e] = lpass + f.dr;
  if (GSC_UNI(hop == f.egress && f.fwd_eg)) fm.departed = 1;
  P.state = F_AFTER_HOP;
  P.c = (int16_t)c;
  P.ret = (int16_t)hop;
  P.pad = (int16_t)e;
  S.procs[pid] = P;
  timeout(S, pid, P.flow, hd);
  if (rel_e >= 0) ledger_push(S, S.h->now + f.duration, rel_e, f.dr);
  (void)K;
}

// DefaultFlowProcessor.process_flow (default_processor.py:14-50) + get_processing_delay.
GSC_HD_CALL void run_process(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P0, const Flow& f) {
  Proc P = P0;
  const int fid = GSC_UNI(P.flow);
  const int Sd = S.d.S;
  const int pstate = GSC_UNI(P.state);
  if (pstate == PR_INIT) {
    const int node = GSC_UNI(f.node);
    const int sf = GSC_UNI(K.chain[GSC_UNI(f.sfc) * kMaxF + GSC_UNI(f.pos)]);
    Flow& fm = S.flows[fid];
    fm.cur_sf = (int16_t)sf;
    if (!GSC_UNI(S.placement[node * Sd + sf])) { proc_return(S, pid, P, 0); return; }
    const double pd = fabs(rng_normal(S, K.pd_mean[sf], K.pd_std[sf]));
    if (GSC_UNI(f.ttl - pd <= 0)) { fm.ttl = 0; proc_return(S, pid, P, 0); return; }
    Stats* st = S.st;
    GSC_ST_LANE0 {
      st_add(&st->num_proc_delays, 1);
      st_add(&st->total_proc_delay, pd);
    }
    fm.e2e = f.e2e + pd;
    fm.ttl = f.ttl - pd;
    if (GSC_UNI(pd == 0.0)) { proc_return(S, pid, P, 0); return; }  // reference: `if not processing_delay`
    P.x = pd;
    P.a = (int16_t)node;
    P.b = (int16_t)sf;
    P.state = PR_AFTER_REQ;
    S.procs[pid] = P;
    const int c = spawn(S, P_REQUEST, RQ_INIT, fid, pid);
    if (c >= 0) { S.procs[c].a = (int16_t)node; S.procs[c].b = (int16_t)sf; }
    return;
  }
  if (pstate == PR_AFTER_REQ) {
    if (!GSC_UNI(P.ret)) { proc_return(S, pid, P, 0); return; }
    S.procs[pid].state = PR_AFTER_WAIT;
    timeout(S, pid, P.flow, P.x);
    return;
  }
  // PR_AFTER_WAIT: spawn finish_processing, return True
  const int c = spawn(S, P_FINISH, FI_INIT, fid, -1);
  if (c >= 0) { S.procs[c].a = P.a; S.procs[c].b = P.b; }
  proc_return(S, pid, P, 1);
  (void)T;
}

// BaseFlowProcessor.request_resources (base_processor.py:51-101).
GSC_HD_CALL void run_request(Env& S, const SimConst& K, int pid, const Proc& P, const Flow& f) {
  if (GSC_UNI(P.state) == RQ_AFTER) { proc_return(S, pid, P, 1); return; }
  const int fid = GSC_UNI(P.flow);
  const int node = GSC_UNI(P.a), sf = GSC_UNI(P.b), Sd = S.d.S;
  double demanded = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
  {  // the node's SF rows loaded by one lane each (one LDS round trip), summed in the serial order
    const int lane = wave_lane();
    int pres = 0;
    double ld = 0.0;
    if (lane < Sd) { pres = S.sf_present[node * Sd + lane]; ld = S.sf_load[node * Sd + lane]; }
    for (int s = 0; s < Sd; ++s)
      if (__builtin_amdgcn_readlane(pres, s)) demanded += readlane_f64(ld, s) + (s == sf ? f.dr : 0.0);
  }
#else
  for (int s = 0; s < Sd; ++s)
    if (GSC_UNI(S.sf_present[node * Sd + s])) demanded += S.sf_load[node * Sd + s] + (s == sf ? f.dr : 0.0);
#endif
  const double cap = S.node_cap[node];
  if (GSC_UNI(!(demanded <= cap))) { proc_return(S, pid, P, 0); return; }
  Flow& fm = S.flows[fid];
  fm.proc_idx = f.proc_idx + 1;
  S.proc_traffic[node * Sd + sf] += f.dr;
  S.sf_load[node * Sd + sf] += f.dr;
  S.node_rem[node] = cap - demanded;
  if (demanded > S.max_usage[node]) S.max_usage[node] = demanded;
  const double ready = S.sf_start[node * Sd + sf] + K.startup[sf];
  if (GSC_UNI(!(ready <= S.h->now))) {
    const double rem = ready - S.h->now;
    if (GSC_UNI(f.ttl - rem <= 0)) { fm.ttl = 0; proc_return(S, pid, P, 0); return; }
    fm.e2e = f.e2e + rem;
    fm.ttl = f.ttl - rem;
    S.procs[pid].state = RQ_AFTER;
    timeout(S, pid, P.flow, rem);
    return;
  }
  proc_return(S, pid, P, 1);
}

// BaseFlowProcessor.finish_processing (base_processor.py:103-135).
GSC_HD_CALL void run_finish(Env& S, const SimConst& K, int pid, const Proc& P, const Flow& f) {
  const int Sd = S.d.S;
  if (GSC_UNI(P.state) == FI_INIT) {
    const int fid = GSC_UNI(P.flow);
    Flow& fm = S.flows[fid];
    const int pos = GSC_UNI(f.pos) + 1;
    fm.pos = (int16_t)pos;
    if (pos == GSC_UNI(K.chain_len[GSC_UNI(f.sfc)])) fm.fwd_eg = 1;
    Proc& pm = S.procs[pid];
    pm.x = f.dr;
    pm.state = FI_AFTER;
    timeout(S, pid, P.flow, f.duration);
    return;
  }
  const int node = GSC_UNI(P.a), sf = GSC_UNI(P.b);
  const double load = S.sf_load[node * Sd + sf] - P.x;
  S.sf_load[node * Sd + sf] = load;
  if (GSC_UNI(load == 0.0 && !S.placement[node * Sd + sf])) S.sf_present[node * Sd + sf] = 0;
  double used = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
  {  // as in run_request: one lane per SF row, serial-order sum
    const int lane = wave_lane();
    int pres = 0;
    double ld = 0.0;
    if (lane < Sd) { pres = S.sf_present[node * Sd + lane]; ld = S.sf_load[node * Sd + lane]; }
    for (int s = 0; s < Sd; ++s)
      if (__builtin_amdgcn_readlane(pres, s)) used += readlane_f64(ld, s);
  }
#else
  for (int s = 0; s < Sd; ++s)
    if (GSC_UNI(S.sf_present[node * Sd + s])) used += S.sf_load[node * Sd + s];
#endif
  S.node_rem[node] = S.node_cap[node] - used;
  proc_return(S, pid, P, 0);
}

// FlowSimulator.init_arrival + DefaultFlowGenerator.generate_flow.
template <bool TLDS = false>
GSC_HD_CALL void run_arrival(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P) {
  const int node = GSC_UNI(P.a);
  const double mean = S.inter_arr[node];
  if (GSC_UNI(mean != mean)) { proc_return(S, pid, P, 0); return; }  // None: arrivals at this node stop
  Header* h = S.h;
  h->total_flow_count++;
  const double inter = K.det_arrival ? mean : exp_from_u01(rng_u01(S), mean);
  double dr, size;
  for (;;) {
    dr = rng_normal(S, K.dr_mean, K.dr_std);
    size = K.det_size ? K.size_shape : pareto_from_u01(rng_u01(S), K.size_shape);  // pareto(a) + 1
    if (GSC_UNI(dr >= 0.0 && size >= 0.0)) break;
  }
  const int sfc = rng_int(S, K.C);
  const int eg = T.n_eg > 0 ? tab<TLDS>(T.egress, rng_int(S, T.n_eg)) : -1;
  const double ttl = K.ttl[rng_int(S, K.n_ttl)];
  const int fid = alloc_flow(S);
  if (fid >= 0) {
    Flow f;
    f.dr = dr;
    f.duration = (size / dr) * 1000.0;
    f.e2e = 0.0;
    f.ttl = ttl;
    f.creation = h->now;
    f.id = h->total_flow_count;
    f.node = (int16_t)node;
    f.ingress = (int16_t)node;
    f.egress = (int16_t)eg;
    f.sfc = (int16_t)sfc;
    f.pos = 0;
    f.cur_sf = -1;
    f.departed = f.fwd_eg = f.dropped = f.proc_idx = 0;
    S.flows[fid] = f;
    Stats* st = S.st;
    GSC_ST_LANE0 {
      st_add(&st->gen, 1);
      st_add(&st->run_gen, 1);
      st_add(&st->active, 1);
    }
    if (spawn(S, P_HANDLE, H_LOOP, fid, -1) < 0) free_flow(S, fid);
  } else {
    h->eid++;  // keep event ids aligned with the oracle even on overflow
  }
  timeout(S, pid, -1, inter);
}

// ResultWriter.begin_writing / write_network_state: the run-window clock.
template <bool BIG = false>
GSC_HD_CALL void run_writer(Env& S, const SimConst& K, const TopoDev& T, int pid, const Proc& P) {
  switch (GSC_UNI(P.state)) {
    case W_BEGIN:
    case W_AFTER:
      respawn_self(S, pid, W_INIT);
      return;
    default:  // W_INIT
#if defined(__HIP_DEVICE_COMPILE__)
      reset_run_metrics<BIG>(S, K, T.n, wave_lane(), 64);
#else
      reset_run_metrics(S, K, T.n, 0, 1);
#endif
      S.procs[pid].state = W_AFTER;
      timeout(S, pid, -1, K.run_duration);
      return;
  }
}

// SimulatorParams.start_mmpp / update_state: 2-state MMPP arrivals.
GSC_HD_CALL void run_mmpp(Env& S, const SimConst& K, const TopoDev& T, int pid) {
  Proc& P = S.procs[pid];
  if (P.state == M_START) {
    P.state = M_AFTER;
    timeout(S, pid, -1, K.run_duration);
    return;
  }
  if (P.state == M_AFTER) {
    respawn_self(S, pid, M_UPDATE);
    return;
  }
  for (int i = 0; i < T.n_ing; ++i) {
    const int v = T.ingress[i];
    int st = S.mmpp_state[v];
    if (rng_u01(S) < K.mmpp_switch[st]) st = 1 - st;
    S.mmpp_state[v] = st;
  }
  for (int i = 0; i < T.n_ing; ++i) S.inter_arr[T.ingress[i]] = K.mmpp_mean[S.mmpp_state[T.ingress[i]]];
  P.state = M_AFTER;
  timeout(S, pid, -1, K.run_duration);
}

// TraceProcessor.process_trace.
GSC_HD_CALL void run_trace(Env& S, const SimConst& K, const TopoDev& T, int pid) {
  Proc& P = S.procs[pid];
  const int i = S.h->trace_index;
  if (P.state == TR_INIT) {
    double w = K.trace_time[i] - S.h->now - 1.0;
    if (w < 0) w = 0;
    P.state = TR_AFTER;
    timeout(S, pid, -1, w);
    return;
  }
  const double mean = K.trace_mean[i];
  if (K.trace_has_node) {
    const int v = K.trace_node[i];
    if (mean != mean) {
      S.inter_arr[v] = mean;
    } else {
      S.inter_arr[v] = mean;
      const double cap = K.trace_cap[i];
      if (cap == cap) S.node_cap[v] = cap;
    }
  } else {
    for (int k = 0; k < T.n_ing; ++k) S.inter_arr[T.ingress[k]] = mean;
  }
  if (i < K.n_trace - 1) {
    S.h->trace_index++;
    respawn_self(S, pid, TR_INIT);  // env.process(process_trace()) ...
    S.h->eid++;                     // ... then this generator returns (completion, no waiter)
  } else {
    proc_return(S, pid, P, 0);
  }
}

// Resume process pid; `fid` = its flow as carried by the event (-1: none).  The process record and
// the flow record are loaded together (one LDS round trip instead of two dependent ones).
#if defined(__HIP_DEVICE_COMPILE__)
// The process record (8 dwords) and the flow record (16 dwords) read with ONE ds_read_b32: lane k < 8
// holds dword k of the process record, lane 8 + j dword j of the flow record; each field is then taken
// from its lane with v_readlane (an SGPR: wave-uniform by construction).  A broadcast ds_read_b128 of
// the same 96 bytes into every lane moves 6 KB through the CU's LDS pipe (64 copies), which the up to
// four simulator waves of a CU queue on.
__device__ __forceinline__ void load_proc_flow(const Env& S, int pid, int fid, Proc& P, Flow& f) {
  static_assert(sizeof(Proc) == 32 && sizeof(Flow) == 64, "record layouts");
  const int lane = wave_lane();
  const uint32_t* pp = reinterpret_cast<const uint32_t*>(S.procs + pid);
  const uint32_t* fp = reinterpret_cast<const uint32_t*>(S.flows + (fid >= 0 ? fid : 0));
  const uint32_t v = lane < 8 ? pp[lane] : fp[(lane - 8) & 15];
  uint32_t w[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) w[k] = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
  __builtin_memcpy(&P, w, 32);
  __builtin_memcpy(&f, w + 8, 64);
}
#endif

template <bool BIG = false, bool TLDS = false>
GSC_HD void dispatch(Env& S, const SimConst& K, const TopoDev& T, int pid, int fid) {
  Proc P;
  Flow f;
#if defined(__HIP_DEVICE_COMPILE__)
  load_proc_flow(S, pid, fid, P, f);
#else
  P = S.procs[pid];
  if (fid >= 0) f = S.flows[fid];
#endif
  if (GSC_UNI(P.flow) != fid) S.h->flags |= FLAG_BAD_STATE;  // event / process flow mismatch
  switch (GSC_UNI(P.type)) {
    case P_HANDLE: run_handle(S, K, T, pid, P, f); break;
    case P_DECIDE: run_decide<BIG>(S, K, T, pid, P, f); break;
    case P_FORWARD: run_forward<BIG, TLDS>(S, K, T, pid, P, f); break;
    case P_PROCESS: run_process(S, K, T, pid, P, f); break;
    case P_REQUEST: run_request(S, K, pid, P, f); break;
    case P_FINISH: run_finish(S, K, pid, P, f); break;
    case P_ARRIVAL: run_arrival<TLDS>(S, K, T, pid, P); break;
    case P_WRITER: run_writer<BIG>(S, K, T, pid, P); break;
    case P_MMPP: run_mmpp(S, K, T, pid); break;
    case P_TRACE: run_trace(S, K, T, pid); break;
    default: S.h->flags |= FLAG_BAD_STATE; break;
  }
}

GSC_HD bool ev_less(const Event& a, const Event& b) { return a.t < b.t || (a.t == b.t && a.key < b.key); }

// Serial event selection (host, and the fallback inside the device loop).
GSC_HD int argmin_event_serial(const Env& S) {
  const int ne = S.h->n_events;
  int best = 0;
  for (int i = 1; i < ne; ++i)
    if (ev_less(S.events[i], S.events[best])) best = i;
  return best;
}

GSC_HD void remove_event(Env& S, int idx) {
  const int last = --S.h->n_events;
  if (idx != last) S.events[idx] = S.events[last];
}

// ------------------------------------------------------------------------------------------------
// Episode init / controller apply / observation + reward epilogue
// ------------------------------------------------------------------------------------------------
// BIG: device kernels with HBM-resident [N, C, S, N] tables -- the schedule table is not used there
// (decisions read the action block) and the WRR counters are reset lazily (reset_run_metrics<BIG>)
template <bool BIG = false>
GSC_HD_CALL void env_init(Env& S, const SimConst& K, const TopoDev& T, int topo, uint32_t seed, int episode,
                          int l0 = 0, int ls = 1) {
  Header* h = S.h;
  const int N = S.d.N, Sd = S.d.S, C = S.d.C, n = T.n;
  const double ewma = S.st->ewma_flows;
  lanes_sync(ls);  // every lane has read the values kept across the reset
  *h = Header{};
  if (l0 == 0) {
    *S.st = Stats{};  // episode_return restarts at 0 (gym's per-episode return, simple_ddpg.py:254)
    S.st->ewma_flows = episode <= 1 ? 1.0 : ewma;
  }
  lanes_sync(ls);
  h->topo = topo;
  h->episode = episode;
  h->n = n;
  h->run_times = 1;
  h->key0 = seed;
  h->key1 = K.same_seed_every_episode ? 0x5eedu : (0x5eedu ^ ((uint32_t)episode * 0x9E3779B9u));
  h->ctr = 0;
  for (int v = l0; v < N; v += ls) {
    const double cap = v < n ? T.cap[v] : 0.0;
    S.node_cap[v] = cap;
    S.node_rem[v] = cap;
    S.inter_arr[v] = 0.0 / 0.0;  // NaN = None
    S.mmpp_state[v] = 0;
  }
  for (int i = l0; i < N * Sd; i += ls) { S.sf_present[i] = 0; S.placement[i] = 0; S.sf_load[i] = 0; S.sf_start[i] = 0; }
  for (int i = l0; i < N * (Sd + 1); i += ls) S.drop_locs[i] = 0;
  if constexpr (!BIG)
    for (int i = l0; i < N * C * Sd * N; i += ls) S.sched[i] = 0.0;
  for (int e = l0; e < S.d.E; e += ls) {
    S.link_rem[e] = e < T.E ? T.edge_cap[e] : 0.0;
    S.link_passed[e] = 0.0;
    S.link_next[e] = 1.0 / 0.0;
  }
  h->flow_top = S.d.flow_cap;
  for (int i = l0; i < S.d.flow_cap; i += ls) S.flow_free[i] = (int16_t)(S.d.flow_cap - 1 - i);
  h->proc_top = S.d.proc_cap;
  h->proc_head = S.d.proc_cap > 0 ? 0 : -1;  // == proc_free[proc_cap - 1]
  for (int i = l0; i < S.d.proc_cap; i += ls) { S.proc_free[i] = (int16_t)(S.d.proc_cap - 1 - i); S.procs[i].type = P_FREE; }
  reset_run_metrics<BIG>(S, K, n, l0, ls);  // ends with lanes_sync
  // reference order: writer, (MMPP), (trace), arrivals; then one env.step()
  spawn(S, P_WRITER, W_BEGIN, -1, -1);
  if (K.use_states) {
    for (int i = 0; i < T.n_ing; ++i) {
      S.mmpp_state[T.ingress[i]] = K.mmpp_init;
      S.inter_arr[T.ingress[i]] = K.mmpp_mean[K.mmpp_init];
    }
    spawn(S, P_MMPP, M_START, -1, -1);
  } else {
    for (int i = 0; i < T.n_ing; ++i) S.inter_arr[T.ingress[i]] = K.inter_arr_mean;
  }
  if (K.n_trace > 0) spawn(S, P_TRACE, TR_INIT, -1, -1);
  for (int i = 0; i < T.n_ing; ++i) {
    const int pid = spawn(S, P_ARRIVAL, A_LOOP, -1, -1);
    if (pid >= 0) S.procs[pid].a = T.ingress[i];
  }
  // DurationController.get_init_state: env.step().  The writer was spawned first (URGENT, the smallest
  // event id at time 0), so that one step is always the writer's W_BEGIN -- run it directly instead of
  // inlining a second copy of every handler into the kernel (the event loop's dispatch is the only one)
  const int idx = argmin_event_serial(S);
  const Event ev = S.events[idx];
  remove_event(S, idx);
  h->now = ev.t;
  if (ev.proc >= 0 && S.procs[ev.proc].type == P_WRITER) {
    const Proc P = S.procs[ev.proc];
    run_writer<BIG>(S, K, T, ev.proc, P);
  } else {
    h->flags |= FLAG_BAD_STATE;
  }
}

// SimulatorWrapper.apply (placement derivation) + DurationController.get_next_state prologue.
// The schedule table S.sched must already hold this step's action.
template <bool BIG = false>
GSC_HD_CALL void controller_prologue(Env& S, const SimConst& K, const TopoDev& T) {
  const int N = S.d.N, Sd = S.d.S, C = S.d.C, n = T.n;
#if defined(__HIP_DEVICE_COMPILE__)
  // lane-parallel over destination nodes: the frontier walk reads each source row with one load per
  // lane, and the next frontier is the ballot of positive weights (== the serial loops below)
  {
    const int lane = wave_lane();
    for (int i = lane; i < N * Sd; i += 64) S.placement[i] = 0;
    lanes_sync(64);
    const bool masks = BIG && n > 64 && pmask_rows(S.d) > 0;  // row bitsets written by sim_pmask_kernel
    for (int c = 0; c < K.C; ++c) {
      uint64_t f[4] = {0, 0, 0, 0};  // node bitset (n <= 256)
      for (int i = 0; i < T.n_ing; ++i) {
        const int v = GSC_UNI(T.ingress[i]);
        if (GSC_UNI(S.inter_arr[v] == S.inter_arr[v])) f[v >> 6] |= 1ull << (v & 63);
      }
      if (masks) {
        // next frontier = OR of the frontier rows' bitsets: one source per lane (all loads of a pass
        // in flight), OR-reduced across the wave; placement from the result
        for (int k = 0; k < K.chain_len[c]; ++k) {
          const int sf = K.chain[c * kMaxF + k];
          uint64_t nf[4] = {0, 0, 0, 0};
          uint64_t w[4] = {0, 0, 0, 0};  // this lane's OR over its sources (all loads in flight)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int src = 64 * q + lane;
            if (src < n && ((f[q] >> lane) & 1)) {
              const uint64_t* m = S.pmask + 4L * ((src * C + c) * Sd + sf);
#pragma unroll
              for (int j = 0; j < 4; ++j) w[j] |= m[j];
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t lo = dpp_red_u32((uint32_t)w[j], 0u, [](uint32_t a, uint32_t b) { return a | b; });
            const uint32_t hi = dpp_red_u32((uint32_t)(w[j] >> 32), 0u, [](uint32_t a, uint32_t b) { return a | b; });
            nf[j] = ((uint64_t)hi << 32) | lo;
          }
          for (int d0 = 0; d0 < n; d0 += 64) {
            const int dst = d0 + lane;
            if (dst < n && ((nf[d0 >> 6] >> lane) & 1)) S.placement[dst * Sd + sf] = 1;
          }
          for (int j = 0; j < 4; ++j) f[j] = nf[j];
        }
        continue;
      }
      for (int k = 0; k < K.chain_len[c]; ++k) {
        const int sf = K.chain[c * kMaxF + k];
        uint64_t nf[4] = {0, 0, 0, 0};
        for (int src = 0; src < n; ++src) {
          if (!((f[src >> 6] >> (src & 63)) & 1)) continue;
          const double* row = S.sched + ((src * C + c) * Sd + sf) * N;
          const float* arow = BIG ? S.act + ((long)(src * K.C + c) * K.F + sf) * K.n_pad : nullptr;
          for (int d0 = 0; d0 < n; d0 += 64) {
            const int dst = d0 + lane;
            const bool pos = dst < n && (BIG ? arow[dst] > 0.f : row[dst] > 0);
            if (pos) S.placement[dst * Sd + sf] = 1;
            nf[d0 >> 6] |= (uint64_t)__ballot(pos);
          }
        }
        for (int j = 0; j < 4; ++j) f[j] = nf[j];
      }
    }
    lanes_sync(64);
    // available_sf rebuild: keep SFs that still carry load, (re)create placed ones
    const double now = S.h->now;
    for (int i = lane; i < n * Sd; i += 64) {
      if (S.sf_present[i] && S.sf_load[i] != 0.0) continue;
      if (S.placement[i]) { S.sf_present[i] = 1; S.sf_load[i] = 0.0; S.sf_start[i] = now; }
      else S.sf_present[i] = 0;
    }
    lanes_sync(64);
    return;
  }
#endif
  for (int i = 0; i < N * Sd; ++i) S.placement[i] = 0;
  // follow positive weights from every active ingress along each chain (add_placement_recursive)
  for (int c = 0; c < K.C; ++c) {
    uint64_t f0 = 0, f1 = 0, f2 = 0, f3 = 0;  // node bitset (n <= 256)
    for (int i = 0; i < T.n_ing; ++i) {
      const int v = T.ingress[i];
      if (S.inter_arr[v] == S.inter_arr[v]) {
        const uint64_t b = 1ull << (v & 63);
        if (v < 64) f0 |= b; else if (v < 128) f1 |= b; else if (v < 192) f2 |= b; else f3 |= b;
      }
    }
    for (int k = 0; k < K.chain_len[c]; ++k) {
      const int sf = K.chain[c * kMaxF + k];
      uint64_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;
      for (int src = 0; src < n; ++src) {
        const uint64_t w = src < 64 ? f0 : (src < 128 ? f1 : (src < 192 ? f2 : f3));
        if (!((w >> (src & 63)) & 1)) continue;
        const double* row = S.sched + ((src * C + c) * Sd + sf) * N;
        for (int dst = 0; dst < n; ++dst) {
          if (row[dst] > 0) {
            S.placement[dst * Sd + sf] = 1;
            const uint64_t b = 1ull << (dst & 63);
            if (dst < 64) n0 |= b; else if (dst < 128) n1 |= b; else if (dst < 192) n2 |= b; else n3 |= b;
          }
        }
      }
      f0 = n0; f1 = n1; f2 = n2; f3 = n3;
    }
  }
  // available_sf rebuild: keep SFs that still carry load, (re)create placed ones
  const double now = S.h->now;
  for (int v = 0; v < n; ++v)
    for (int s = 0; s < Sd; ++s) {
      const int i = v * Sd + s;
      if (S.sf_present[i] && S.sf_load[i] != 0.0) continue;
      if (S.placement[i]) { S.sf_present[i] = 1; S.sf_load[i] = 0.0; S.sf_start[i] = now; }
      else S.sf_present[i] = 0;
    }
}

GSC_HD void schedule_stop(Env& S, const SimConst& K) {
  const double T_end = K.run_duration * S.h->run_times;
  push_event(S, S.h->now + (T_end - S.h->now), 0u, kStopProc, (int16_t)-1);
}

// Host / serial event loop until the stop event.
GSC_HD void run_until_stop_serial(Env& S, const SimConst& K, const TopoDev& T) {
  for (;;) {
    if (S.h->n_events <= 0) { S.h->flags |= FLAG_BAD_STATE; return; }
    const int idx = argmin_event_serial(S);
    const Event ev = S.events[idx];
    remove_event(S, idx);
    S.h->now = ev.t;
    S.h->cur_key = ev.key;
    if (ev.proc == kStopProc) return;
    dispatch(S, K, T, ev.proc, ev.flow);
  }
}

// Observation [n_pad, n_obs] (float32, max-normalised), reward and per-run stats.
GSC_HD float clip01(float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); }

GSC_HD float obs_feature(const Env& S, const SimConst& K, int q, int v) {
  const int Sd = S.d.S, C = S.d.C;
  if (q == 0) {  // ingress traffic of the chain's first SF (the last SFC with traffic wins, as in the reference)
    float t = 0.f;
    for (int c = 0; c < K.C; ++c) {
      bool any = false;
      for (int s = 0; s < Sd; ++s) any |= S.requested[(v * C + c) * Sd + s] != 0.0;
      if (any) t = (float)S.requested[(v * C + c) * Sd + K.chain[c * kMaxF]];
    }
    return t;
  }
  const double cap = S.node_cap[v];
  if (q == 2) return (float)cap;
  double use = 0.0;
  for (int s = 0; s < Sd; ++s) use += S.proc_traffic[v * Sd + s];
  return cap == 0.0 ? 1.f : (float)(use / cap);
}

GSC_HD_CALL void write_obs(const Env& S, const SimConst& K, const TopoDev& T, float* obs) {
  const int n = T.n;
  for (int j = 0; j < K.n_obs; ++j) {
    const int q = K.obs_feat[j];
    float mx = 0.f;
    for (int v = 0; v < n; ++v) {
      const float x = obs_feature(S, K, q, v);
      mx = (v == 0 || x > mx) ? x : mx;
    }
    const float den = mx + 1e-3f;
    for (int v = 0; v < K.n_pad; ++v) obs[v * K.n_obs + j] = v < n ? clip01(obs_feature(S, K, q, v) / den) : 0.f;
  }
}

// End of a run window: the window's mean path delay (the reference updates it at every path; nothing
// reads it inside the window, so it is derived once here from the window's totals)
GSC_HD void finish_run_stats(Env& S) {
  Stats* st = S.st;
  st->run_avg_path_delay = st->run_gen > 0 ? st->run_total_path_delay / st->run_gen : 0.0;
}

GSC_HD_CALL float compute_reward(Env& S, const SimConst& K, const TopoDev& T) {
  Stats* h = S.st;
  const int succ = h->run_processed, drop = h->run_dropped, Sd = K.S, n = T.n;  // real SF count (dims may be padded)
  double succ_ratio = 0.0, fr = 0.0;
  if (succ + drop > 0) {
    succ_ratio = (double)succ / (succ + drop);
    fr = (double)(succ - drop) / (succ + drop);
  }
  const double diam = K.diameter > 0 ? K.diameter : T.diameter;
  const double avg = succ > 0 ? h->run_e2e / succ : 0.0;
  const double delay = avg > K.min_delay ? avg : K.min_delay;
  double dr;
  if (succ_ratio == 0.0) dr = -1.0;
  else {
    dr = ((K.min_delay - delay) / diam) + 1.0;
    dr = dr < -1 ? -1 : (dr > 1 ? 1 : dr);
  }
  double used = 0.0, inst = 0.0;
  for (int v = 0; v < n; ++v) {
    int cnt = 0;
    for (int s = 0; s < Sd; ++s) cnt += S.placement[v * S.d.S + s];
    inst += cnt;
    if (cnt > 0) used += Sd > 1 ? ((double)(cnt - 1) / (Sd - 1)) * 0.5 + 0.5 : 1.0;
  }
  double nr = 2 * (-used / n) + 1;
  double ir = 2 * (-inst / ((double)n * Sd)) + 1;
  switch (K.objective) {
    case OBJ_PRIO_FLOW: {
      nr = ir = 0;
      double target = K.target_success;
      if (target != target) {
        target = 0.9 * h->ewma_flows;
        h->ewma_flows = 0.5 * succ_ratio + 0.5 * h->ewma_flows;
      }
      if (succ_ratio < target) dr = -1;
      break;
    }
    case OBJ_SOFT_DEADLINE:
      nr = ir = 0;
      if (delay > K.soft_deadline) fr = -1;
      else {
        dr = -K.soft_deadline / diam;
        dr = dr < -1 ? -1 : (dr > 1 ? 1 : dr);
      }
      break;
    case OBJ_SOFT_DEADLINE_EXP: {
      fr = nr = ir = 0;
      double util = 1.0;
      if (delay > K.soft_deadline) {
        util = -log10_cold((1.0 / K.dropoff) * (delay - K.soft_deadline));
        util = util < 0 ? 0 : (util > 1 ? 1 : util);
      }
      dr = succ_ratio * util;
      break;
    }
    default:
      fr *= K.w_flow; dr *= K.w_delay; nr *= K.w_node; ir *= K.w_inst;
  }
  return (float)(fr + dr + nr + ir);
}

GSC_HD void write_stats(const Env& S, float* st) {
  const Stats* h = S.st;
  const Header* hc = S.h;
  st[0] = (float)h->run_processed;
  st[1] = (float)h->run_dropped;
  st[2] = (float)h->run_gen;
  st[3] = (float)(h->run_processed > 0 ? h->run_e2e / h->run_processed : 0.0);
  st[4] = (float)h->processed;
  st[5] = (float)h->dropped;
  st[6] = (float)h->gen;
  st[7] = (float)h->active;
  st[8] = (float)h->drop_reason[0];
  st[9] = (float)h->drop_reason[1];
  st[10] = (float)h->drop_reason[2];
  st[11] = (float)h->drop_reason[3];
  st[12] = (float)hc->flags;
  st[13] = (float)hc->max_events;
  st[14] = (float)hc->max_procs;
  st[15] = (float)hc->max_flows;
}

// Copy this step's (post-processed) action block into the schedule table.
template <bool BIG = false>
GSC_HD void load_action(Env& S, const SimConst& K, const TopoDev& T, const float* act, int lane, int nlanes) {
  const int N = S.d.N, Sd = S.d.S, C = S.d.C, n = T.n, P = K.n_pad;
#if defined(__HIP_DEVICE_COMPILE__)
  // BIG (HBM-resident tables): nothing to copy -- decisions and the placement walk read the action block
  // itself (Env::act) and the destination bitsets of large topologies come from sim_pmask_kernel
  if constexpr (BIG) return;
#endif
  const int total = n * C * Sd * n;
  for (int i = lane; i < total; i += nlanes) {
    const int dst = i % n;
    int r = i / n;
    const int sf = r % Sd; r /= Sd;
    const int c = r % C;
    const int src = r / C;
    S.sched[((src * C + c) * Sd + sf) * N + dst] = (double)act[((src * K.C + c) * K.F + sf) * P + dst];
  }
}

}  // namespace gsc
