"""Batched coord-sim: E environments stepped in lockstep by one native launch per step.

On a GPU every environment is one 64-lane wave (state staged in LDS); on CPU the same C++ core
runs on host threads (used by the CPU test-suite and for differential checks against the scalar
oracle in :mod:`gsc_amd.coordsim`).

Action layout (reference ``EnvironmentLimits.scheduling_shape``): ``[n_pad, C, F, n_pad]``
flattened, weights already thresholded/normalised.  Observation: ``[E, n_pad, n_obs]`` node
features (ingress traffic, node load, node capacity; each max-normalised with +1e-3).

Documented deviations from the reference (see ``docs/DEVIATIONS.md``):
* per-env Philox RNG streams (reference: global NumPy/Python RNGs reseeded each episode, Q4);
  ``same_seed_every_episode`` reproduces the reference's identical-episode behaviour;
* only the default plugin set (DefaultFlowGenerator/ListFlowGenerator, DefaultDecisionMaker,
  DefaultFlowForwarder, DefaultFlowProcessor, DurationController) and identity resource
  functions run natively — other plugins run on the scalar oracle;
* MMPP state and trace-modified node capacities are reset at every episode start.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from gsc_amd.coordsim import reader
from gsc_amd.coordsim.reader import Topology
from gsc_amd.native import load as load_native

OBS_FEATURES = {"ingress_traffic": 0, "node_load": 1, "node_cap": 2}
OBJECTIVES = {"prio-flow": 0, "soft-deadline": 1, "soft-deadline-exp": 2, "weighted": 3}
NATIVE_PLUGINS = {
    "flow_generator_class": {"DefaultFlowGenerator", "ListFlowGenerator"},
    "flow_forwarder_class": {"DefaultFlowForwarder"},
    "flow_processor_class": {"DefaultFlowProcessor"},
    "decision_maker_class": {"DefaultDecisionMaker"},
    "controller_class": {"DurationController"},
}
STAT_NAMES = ["run_succ", "run_drop", "run_gen", "run_avg_e2e", "succ", "drop", "gen", "active", "drop_ttl",
              "drop_decision", "drop_link", "drop_node", "flags", "max_events", "max_procs", "max_flows"]


@dataclass
class SimStepOut:
    obs: torch.Tensor        # [E, n_pad, n_obs] observation for the next action (reset obs where done)
    next_obs: torch.Tensor   # [E, n_pad, n_obs] observation reached (terminal obs where done)
    reward: torch.Tensor     # [E]
    done: torch.Tensor       # [E] bool
    stats: torch.Tensor      # [E, 16] see STAT_NAMES
    ep_return: torch.Tensor  # [E] finished-episode return (valid where done)


def sim_config_from_files(sim_config: dict, sfc_list: dict, sf_list: dict, agent_config: dict,
                          trace_rows: Optional[list] = None, node_index: Optional[dict] = None):
    """Translate reference YAML configs into the native ``SimConst`` dictionary (host arrays kept separately)."""
    for key, allowed in NATIVE_PLUGINS.items():
        name = sim_config.get(key)
        if name is not None and name not in allowed:
            raise ValueError(f"{key}={name} is not supported by the batched simulator (use the scalar oracle)")
    sf_names = list(sf_list.keys())
    sfc_names = list(sfc_list.keys())
    for sf in sf_names:
        if sf_list[sf].get("resource_function_id", "default") != "default":
            raise ValueError(f"SF {sf}: custom resource functions run only on the scalar oracle")
    F = max(len(v) for v in sfc_list.values())
    chain = [[sf_names.index(sf) for sf in sfc_list[c]] for c in sfc_names]
    det_arr = sim_config.get("deterministic", None)
    det_size = sim_config.get("deterministic", None)
    det_arr = sim_config.get("deterministic_arrival", det_arr)
    det_size = sim_config.get("deterministic_size", det_size)
    if det_arr is None or det_size is None:
        raise ValueError("'deterministic_arrival' or 'deterministic_size' are not set in simulator config.")
    use_states = bool(sim_config.get("use_states", False))
    mm_mean, mm_switch, mm_init = [0.0, 0.0], [0.0, 0.0], 0
    if use_states:
        names = list(sim_config["states"].keys())
        if len(names) != 2:
            raise ValueError("MMPP needs exactly two states")
        mm_mean = [float(sim_config["states"][k]["inter_arr_mean"]) for k in names]
        mm_switch = [float(sim_config["states"][k]["switch_p"]) for k in names]
        mm_init = names.index(sim_config["init_state"])
    obj = agent_config.get("objective", "weighted")
    target = agent_config.get("target_success")
    diam = agent_config.get("network_diameter", 15)
    cfg = dict(
        C=len(sfc_names), S=len(sf_names), F=F, chain=chain,
        pd_mean=[float(sf_list[s]["processing_delay_mean"]) for s in sf_names],
        pd_std=[float(sf_list[s]["processing_delay_stdev"]) for s in sf_names],
        startup=[float(sf_list[s]["startup_delay"]) for s in sf_names],
        run_duration=float(sim_config["run_duration"]), det_arrival=int(bool(det_arr)), det_size=int(bool(det_size)),
        dr_mean=float(sim_config["flow_dr_mean"]), dr_std=float(sim_config["flow_dr_stdev"]),
        size_shape=float(sim_config["flow_size_shape"]), ttl=[float(t) for t in sim_config["ttl_choices"]],
        inter_arr_mean=float(sim_config["inter_arrival_mean"]), use_states=int(use_states), mmpp_init=mm_init,
        mmpp_mean=mm_mean, mmpp_switch=mm_switch,
        obs_feat=[OBS_FEATURES[o] for o in agent_config.get("observation_space", ["ingress_traffic"])],
        objective=OBJECTIVES[obj],
        w_flow=float(agent_config.get("flow_weight", 0) or 0), w_delay=float(agent_config.get("delay_weight", 0) or 0),
        w_node=float(agent_config.get("node_weight", 0) or 0), w_inst=float(agent_config.get("instance_weight", 0) or 0),
        target_success=(math.nan if target in (None, "auto") else float(target)),
        soft_deadline=float(agent_config.get("soft_deadline") or 0.0), dropoff=float(agent_config.get("dropoff") or 1.0),
        min_delay=float(sum(sf_list[s]["processing_delay_mean"] for s in sf_names)),
        diameter=(-1.0 if diam == "auto" else float(diam)),
        episode_steps=int(agent_config.get("episode_steps", 200)),
    )
    if obj == "prio-flow" and target is None:
        raise ValueError("prio-flow objective needs target_success")
    trace = None
    if trace_rows:
        has_node = "node" in trace_rows[0]
        t_time = np.asarray([float(r["time"]) for r in trace_rows], np.float64)
        t_node = np.asarray([node_index[r["node"]] if has_node else -1 for r in trace_rows], np.int16)
        t_mean = np.asarray([math.nan if r["inter_arrival_mean"] == "None" else float(r["inter_arrival_mean"])
                             for r in trace_rows], np.float64)
        t_cap = np.asarray([float(r["cap"]) if "cap" in r and r["cap"] not in (None, "") else math.nan
                            for r in trace_rows], np.float64)
        trace = dict(time=t_time, node=t_node, mean=t_mean, cap=t_cap, has_node=int(has_node))
    return cfg, trace, sf_names, sfc_names


def _default_caps(topos: Sequence[Topology], cfg: dict, trace: Optional[dict] = None) -> dict:
    """Pool capacities sized from the arrival rate (flows alive within one TTL), with margin."""
    max_ing = max(len(t.ingress) for t in topos)
    mean = cfg["inter_arr_mean"]
    if cfg["use_states"]:
        mean = min(mean, min(cfg["mmpp_mean"]))
    ttl = max(cfg["ttl"])
    # flows alive at once <= arrivals within one TTL (every flow ends by its TTL): per ingress
    # ttl / mean, x 2.5 for Poisson bursts, + 8.  Measured peaks on the shipped configs (random
    # schedules) are >= 4x below this (tests/test_batched_sim_diff.py::test_default_caps_headroom); pools
    # are LDS (a 50-node env's pools fit two envs per CU)
    burst = 1.0 if cfg["det_arrival"] else 2.5
    rate = burst / max(mean, 1e-3)  # arrivals per ms and ingress, with burst margin
    if trace is not None and len(trace["mean"]):
        tm = np.asarray(trace["mean"], np.float64)
        tm = tm[np.isfinite(tm)]
        if len(tm):  # a trace sets the inter-arrival means: its busiest row (already a peak) may exceed the margin
            rate = max(rate, 1.0 / max(float(tm.min()), 1e-3))
    mean = burst / rate
    per_node = ttl * rate + 8
    flows = int(min(4096, max(64, max_ing * per_node)))
    # processes and link returns outlive their flow by its duration (finish_processing and
    # return_link_resources hold `duration` = size / dr * 1000 ms): the arrivals within one duration
    # hold up to F finish processes and one return per hop each
    dr_low = max(cfg["dr_mean"] - 2.0 * cfg["dr_std"], 0.1 * cfg["dr_mean"], 1e-6)
    if cfg["det_size"]:
        size = cfg["size_shape"]
    else:  # Pareto(shape) + 1: mean shape / (shape - 1); heavy tails are capped by the pool limits below
        a = cfg["size_shape"]
        size = a / (a - 1.0) if a > 1.0 else 8.0
    dur = size / dr_low * 1000.0
    hold = max_ing * (dur / max(mean, 1e-3) * burst + 4) if dur > 1.0 else 0.0
    hops = max(t.max_hops for t in topos)
    # the pending-event queue lives in VGPRs on the device (64 per set); observed peaks on the reference
    # configs are 30-60 events, so 128 leaves 2x headroom (overflow is flagged, never silent)
    # pending link returns: one per hop a flow took within its duration -- long paths (200 nodes:
    # 12 hops) hold several per flow
    # pending events: the register queue holds 64 per set (csrc/sim/sim_kernels.hip RegQueue); measured peaks
    # are 0.25-0.4 x the flow capacity (28 of 72 on sample_config, 72 of 288 at 200 nodes).  One set (64) for
    # sample_config measured slower than two, 2.25 vs 2.16 ms/step on the bench's 64 CUs (the step kernel's
    # code layout, not its instruction count, decides there), so 128 stays the floor
    ev = 128 if max_ing <= 8 else 256
    ev = int(os.environ.get("GSC_SIM_EVENT_CAP", ev))
    return dict(flow_cap=flows, proc_cap=int(min(32000, 2 * flows + 32 + cfg["F"] * hold)),
                event_cap=ev,
                rel_cap=int(min(16384, 2 * flows * max(1.0, hops / 4) + hops * hold)))


class BatchedSimulator:
    def __init__(self, topologies: List[Topology], sfc_list: dict, sf_list: dict, sim_config: dict,
                 agent_config: dict, num_envs: int, device="cpu", seed: int = 0, n_pad: Optional[int] = None,
                 caps: Optional[dict] = None, same_seed_every_episode: bool = False, trace_rows=None,
                 host_threads: int = 8, topo_init: Optional[Sequence[int]] = None):
        self.native = load_native()
        self.device = torch.device(device)
        self.is_device = self.device.type == "cuda"
        self.topologies = list(topologies)
        self.E = int(num_envs)
        N = max(t.n for t in self.topologies)
        self.n_pad = int(n_pad if n_pad is not None else agent_config.get("max_nodes", 24))
        if self.n_pad < N:
            raise ValueError(f"n_pad={self.n_pad} < largest topology ({N} nodes)")
        node_index = {nid: i for i, nid in enumerate(self.topologies[0].node_ids)}
        cfg, trace, self.sf_names, self.sfc_names = sim_config_from_files(sim_config, sfc_list, sf_list,
                                                                           agent_config, trace_rows, node_index)
        cfg["n_pad"] = self.n_pad
        cfg["same_seed_every_episode"] = int(same_seed_every_episode)
        self.cfg = cfg
        self.C, self.S, self.F = cfg["C"], cfg["S"], cfg["F"]
        self.n_obs = len(cfg["obs_feat"])
        self.action_dim = self.n_pad * self.C * self.F * self.n_pad
        self.episode_steps = cfg["episode_steps"]
        dev = self.device
        # trace tables
        keep = []
        if trace is None:
            trace = dict(time=np.zeros(1), node=np.zeros(1, np.int16), mean=np.zeros(1), cap=np.zeros(1), has_node=0)
            cfg["n_trace"] = 0
        else:
            cfg["n_trace"] = len(trace["time"])
        cfg["trace_has_node"] = trace["has_node"]
        for k in ("time", "node", "mean", "cap"):
            t = torch.from_numpy(np.ascontiguousarray(trace[k])).to(dev)
            keep.append(t)
            cfg[f"trace_{k}"] = t.data_ptr()
        # topology tables
        topo_dicts = []
        for t in self.topologies:
            # edge of hop k on the shortest path i -> j (from node k-1 of the path, or i), so the
            # forwarder reads a hop's node and edge in parallel instead of one after the other
            pn = np.asarray(t.path_nodes)
            prev = np.concatenate([np.broadcast_to(np.arange(t.n)[:, None, None], (t.n, t.n, 1)), pn[:, :, :-1]], axis=2)
            pedges = np.where(pn >= 0, np.asarray(t.edge_id)[prev.clip(0), pn.clip(0)], -1)
            # delay of each hop (== path_delay[previous node][hop]): read with the hop's node / edge when the
            # topology tables stay in HBM (200-node topologies) instead of after them
            phd = np.where(pn >= 0, np.asarray(t.path_delay)[prev.clip(0), pn.clip(0)], 0.0).astype(np.float64)
            tens = dict(cap=torch.from_numpy(t.node_cap.astype(np.float64)),
                        pdelay=torch.from_numpy(np.ascontiguousarray(t.path_delay.reshape(-1))),
                        plen=torch.from_numpy(t.path_len.reshape(-1).astype(np.int16)),
                        pnodes=torch.from_numpy(t.path_nodes.reshape(-1).astype(np.int16)),
                        pedges=torch.from_numpy(pedges.reshape(-1).astype(np.int16)),
                        phd=torch.from_numpy(np.ascontiguousarray(phd.reshape(-1))),
                        edge_id=torch.from_numpy(t.edge_id.reshape(-1).astype(np.int16)),
                        edge_cap=torch.from_numpy(np.ascontiguousarray(t.edge_cap) if t.num_edges else np.zeros(1)),
                        ingress=torch.from_numpy(t.ingress.astype(np.int16) if len(t.ingress) else np.zeros(1, np.int16)),
                        egress=torch.from_numpy(t.egress.astype(np.int16) if len(t.egress) else np.zeros(1, np.int16)))
            d = dict(n=t.n, E=t.num_edges, H=t.max_hops, n_ing=len(t.ingress), n_eg=len(t.egress),
                     diameter=float(t.diameter))
            for k, v in tens.items():
                v = v.contiguous().to(dev)
                keep.append(v)
                d[k] = v.data_ptr()
            topo_dicts.append(d)
        self._keep = keep
        caps = dict(caps or _default_caps(self.topologies, cfg, trace if cfg["n_trace"] else None))
        dims = dict(N=N, S=self.S, C=self.C, E=max(1, max(t.num_edges for t in self.topologies)), **caps)
        self.dims = dims
        self.ctx = self.native.SimContext(dims, cfg, topo_dicts, self.is_device, host_threads)
        self.state_bytes = int(self.ctx.state_bytes)
        self.states = torch.zeros((self.E, self.state_bytes), dtype=torch.uint8, device=dev)
        g = np.random.default_rng(seed)
        self.seeds = torch.from_numpy(g.integers(1, 2**31 - 1, size=self.E).astype(np.uint32).view(np.int32)).to(dev)
        init = np.zeros(self.E, np.int32) if topo_init is None else np.asarray(topo_init, np.int32)
        self.topo_next = torch.from_numpy(init).to(dev)
        ob = (self.E, self.n_pad, self.n_obs)
        self.obs = torch.zeros(ob, dtype=torch.float32, device=dev)
        self.next_obs = torch.zeros(ob, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(self.E, dtype=torch.float32, device=dev)
        self.done = torch.zeros(self.E, dtype=torch.uint8, device=dev)
        self.stats = torch.zeros((self.E, self.native.SIM_NUM_STATS), dtype=torch.float32, device=dev)
        self.ep_return = torch.zeros(self.E, dtype=torch.float32, device=dev)
        # output buffer sets for step(buffer_set=k): set 0 is the attributes above; set 1 lets a caller
        # read step t's outputs (replay insert) while step t+1 already writes its own
        self._out_sets = [(self.obs, self.next_obs, self.reward, self.done, self.stats, self.ep_return),
                          tuple(torch.zeros_like(t) for t in (self.obs, self.next_obs, self.reward, self.done,
                                                               self.stats, self.ep_return))]
        self.topo_cur = self.topo_next.clone()
        self.prof = None

    # ------------------------------------------------------------------------------------------
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.is_device else 0

    def set_topologies(self, topo_ids) -> None:
        """Topology index used by each env at its next reset (network scheduler)."""
        t = torch.as_tensor(topo_ids, dtype=torch.int32)
        if t.numel() == 1:
            t = t.expand(self.E)
        self.topo_next.copy_(t.to(self.device))

    def reset(self) -> torch.Tensor:
        self.ctx.reset(self.states.data_ptr(), self.topo_next.data_ptr(), self.seeds.data_ptr(),
                       self.obs.data_ptr(), self.E, self._stream())
        self.topo_cur.copy_(self.topo_next)
        return self.obs

    def enable_profiling(self, on: bool = True) -> None:
        """Accumulate per-env cycle counters in ``self.prof``: [E, 4] (event selection / handlers / merge / events)
        then [E, 64, 2] handler cycles / dispatches per (process type, resume state)."""
        self.prof = torch.zeros(self.E * 4 + self.E * 128, dtype=torch.int64, device=self.device) if on else None

    def pmask_target(self) -> Optional[tuple]:
        """(base, stride, C, F, Cd, Sd, N) for the exploration kernel to write the step kernel's destination bitsets
        (topologies beyond 64 nodes with HBM-resident tables), or None when the kernel does not read them.  The
        block holds rows for the N source nodes of the largest topology only; the kernel skips action rows of
        sources >= N (n_pad > N)."""
        lay = self.ctx.pmask_layout if self.is_device else None
        if lay is None:
            return None
        off, Cd, Sd = lay
        return (self.states.data_ptr() + int(off), self.state_bytes, self.C, self.F, int(Cd), int(Sd),
                int(self.dims["N"]))

    def step(self, actions: torch.Tensor, buffer_set: int = 0, obs_out: Optional[torch.Tensor] = None,
             pmask_ready: bool = False) -> SimStepOut:
        """One lockstep step of every env.  ``obs_out``: write the next action's observations there
        instead of the buffer set's own ``obs`` (the trainer's rotating observation buffers).  ``pmask_ready``:
        the producer of ``actions`` already wrote the destination bitsets (``pmask_target``)."""
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.dim() != 2 or actions.shape[0] != self.E or actions.shape[1] < self.action_dim:
            raise ValueError(f"actions must be [E={self.E}, >= {self.action_dim}], got {tuple(actions.shape)}")
        obs, next_obs, reward, done_u8, stats, ep_return = self._out_sets[buffer_set]
        if obs_out is not None:
            assert obs_out.shape == obs.shape and obs_out.dtype == obs.dtype and obs_out.is_contiguous()
            assert obs_out.device.type == self.device.type
            obs = obs_out
        # envs that finish are reset onto their scheduled topology: the kernel updates topo_cur there
        self.ctx.step(self.states.data_ptr(), self.topo_next.data_ptr(), self.seeds.data_ptr(), actions.data_ptr(),
                      actions.shape[1], obs.data_ptr(), next_obs.data_ptr(), reward.data_ptr(),
                      done_u8.data_ptr(), stats.data_ptr(), ep_return.data_ptr(), self.E, self._stream(),
                      self.prof.data_ptr() if (self.prof is not None and self.is_device) else 0,
                      self.topo_cur.data_ptr(), bool(pmask_ready))
        done = done_u8.view(torch.bool)  # 0/1 bytes: zero-copy
        return SimStepOut(obs, next_obs, reward, done, stats, ep_return)

    def check_flags(self) -> int:
        flags = int(max(t[4][:, 12].max() for t in self._out_sets).item())
        if flags:
            raise RuntimeError(f"batched simulator overflow/bad state flags={flags} (caps {self.dims}; bits: 1 flows, "
                               "2 processes, 4 events, 8 bad state, 16 link releases); increase the capacities")
        return flags

    def action_mask(self, topo_index: int = 0) -> torch.Tensor:
        n = self.topologies[topo_index].n
        m = torch.zeros((self.n_pad, self.C, self.F, self.n_pad), dtype=torch.float32)
        m[:n, :, :, :n] = 1
        return m.reshape(-1)


def load_batched_from_paths(network_files: Sequence[str], service_file: str, sim_config_file: str,
                            agent_config: dict, num_envs: int, device="cpu", seed=0, **kw) -> BatchedSimulator:
    sim_cfg = reader.get_config(sim_config_file)
    topos = [reader.load_topology(f, sim_cfg) for f in network_files]
    trace_rows = None
    if "trace_path" in sim_cfg:
        from gsc_amd.coordsim.simulator import resolve_trace_path
        trace_rows = reader.get_trace(resolve_trace_path(sim_cfg["trace_path"], sim_config_file))
    return BatchedSimulator(topos, reader.get_sfc(service_file), reader.get_sf(service_file), sim_cfg, agent_config,
                            num_envs, device=device, seed=seed, trace_rows=trace_rows, **kw)
