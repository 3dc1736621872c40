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
#include <thread>
#include <vector>

#include "../common.h"
#include "sim_core.h"

namespace py = pybind11;

namespace gsc {

constexpr long kMaxEventsPerStep = 4000000;  // runaway guard (no GPU hang on a bad state)

struct SimArgs {
  char* states;
  long state_bytes;
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
};

GSC_HD void step_epilogue(Env& S, const SimArgs& a, int env) {
  const SimConst& K = a.K;
  const TopoDev& T = a.topos[S.h->topo];
  const long ostride = (long)K.n_pad * K.n_obs;
  S.h->run_times++;
  const float r = compute_reward(S, K, T);
  write_stats(S, a.stats + (long)env * kNumStats);
  write_obs(S, K, T, a.next_obs + env * ostride);
  a.reward[env] = r;
  S.h->episode_return += r;
  S.h->run_count++;
  if (S.h->run_count >= K.episode_steps) {
    a.done[env] = 1;
    a.ep_return[env] = (float)S.h->episode_return;
    const int topo = a.topo_next[env];
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
  S.h->episode_return = 0.0;
  S.h->ewma_flows = 1.0;
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

__device__ __forceinline__ int argmin_event_wave(const Env& S, int lane) {
  const int ne = S.h->n_events;
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

__device__ __forceinline__ void device_step_env(const SimArgs& a, char* base, int env, int lane) {
  Env S(base, a.L, a.D);
  const TopoDev& T = a.topos[S.h->topo];
  load_action(S, a.K, T, a.actions + (long)env * a.action_stride, lane, 64);
  __syncthreads();
  if (lane == 0) {
    controller_prologue(S, a.K, T);
    schedule_stop(S, a.K);
  }
  __syncthreads();
  for (long it = 0;; ++it) {
    const int idx = argmin_event_wave(S, lane);
    if (idx < 0 || it > kMaxEventsPerStep) {
      if (lane == 0) S.h->flags |= FLAG_BAD_STATE;
      break;
    }
    const Event ev = S.events[idx];
    __syncthreads();
    if (lane == 0) {
      remove_event(S, idx);
      S.h->now = ev.t;
      if (ev.proc != kStopProc) dispatch(S, a.K, T, ev.proc);
    }
    __syncthreads();
    if (ev.proc == kStopProc) break;
  }
  __syncthreads();
  if (lane == 0) step_epilogue(S, a, env);
  __syncthreads();
}

__global__ __launch_bounds__(64) void sim_step_kernel(SimArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  char* g = a.states + (long)env * a.state_bytes;
  if (a.use_lds) {
    copy16(smem, g, a.state_bytes, lane);
    __syncthreads();
    device_step_env(a, smem, env, lane);
    copy16(g, smem, a.state_bytes, lane);
  } else {
    device_step_env(a, g, env, lane);
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
  step_epilogue(S, a, env);
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
      use_lds_ = L_.total <= max_lds;
      if (use_lds_ && L_.total > 65536)
        GSC_HIP_CHECK(hipFuncSetAttribute((const void*)sim_step_kernel,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, L_.total));
    }
  }
  ~SimContext() {
    if (dev_topos_) (void)hipFree(dev_topos_);
  }

  long state_bytes() const { return L_.total; }
  bool use_lds() const { return use_lds_; }

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
            uintptr_t ep_return, int E, uintptr_t stream) {
    SimArgs a = args(states, topo_next, seeds, actions, action_stride, obs, next_obs, reward, done, stats,
                     ep_return, E);
    if (device_) {
      const size_t lds = use_lds_ ? (size_t)L_.total : 0;
      hipLaunchKernelGGL(sim_step_kernel, dim3(E), dim3(64), lds, stream_of(stream), a);
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
    a.use_lds = use_lds_ ? 1 : 0;
    return a;
  }

  void fill_const(py::dict c) {
    SimConst& K = K_;
    K = SimConst{};
    K.C = c["C"].cast<int>();
    K.S = c["S"].cast<int>();
    K.F = c["F"].cast<int>();
    GSC_CHECK(K.C <= kMaxC && K.S <= kMaxS && K.F <= kMaxF, "too many SFCs / SFs");
    GSC_CHECK(K.C == D_.C && K.S == D_.S, "config/dims mismatch");
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
  bool use_lds_ = false;
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
      .def("reset", &SimContext::reset)
      .def("step", &SimContext::step);
  m.attr("SIM_NUM_STATS") = kNumStats;
  m.attr("SIM_HEADER_BYTES") = (int)sizeof(Header);
}

}  // namespace gsc
