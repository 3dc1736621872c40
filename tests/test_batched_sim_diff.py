"""Differential tests: native batched simulator (host path) vs the scalar SimPy-semantics oracle.

Deterministic configurations must agree step by step (success/drop/generated counts, reward,
observation) for arbitrary post-processed schedules; this pins the event-ordering emulation.
"""
import numpy as np
import pytest
import torch
import yaml

from gsc_amd.envs import GymEnv, threshold_normalize
from gsc_amd.sim.batched import load_batched_from_paths
from tests.conftest import cfg_path

ABC = cfg_path("service_functions", "abc.yaml")
AB = cfg_path("service_functions", "ab.yaml")
SAMPLE = cfg_path("config", "simulator", "sample_config.yaml")
NETS = {
    "abilene": cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"),
    "abilene_cap0_2": cfg_path("networks", "abilene", "abilene-in4-rand-cap0-2.graphml"),
    "triangle": cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml"),
    "line": cfg_path("networks", "line", "line-in1-cap1-delay10.graphml"),
    "bteurope": cfg_path("networks", "bteurope", "bteurope-in4-rand-cap0-2.graphml"),
}


def agent_cfg():
    return yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))


def random_actions(rng, steps, n, C, F, pad=24, density=0.35):
    acts = []
    for _ in range(steps):
        a = np.zeros((pad, C, F, pad))
        raw = rng.random((n, C, F, n))
        raw[rng.random((n, C, F, n)) > density] = 0.0
        a[:n, :, :, :n] = raw
        a = threshold_normalize(a.reshape(-1), pad, 0.1, passes=2).astype(np.float32)
        acts.append(a)
    return acts


@pytest.mark.parametrize("net,svc,steps", [("abilene", ABC, 60), ("abilene_cap0_2", ABC, 40),
                                           ("triangle", ABC, 40), ("line", AB, 40), ("bteurope", ABC, 30)])
def test_native_matches_oracle_per_step(net, svc, steps):
    cfg = agent_cfg()
    cfg["episode_steps"] = steps + 5
    path = NETS[net]
    sched = {"training_network_files": [path], "inference_network": path, "period": 10}
    env = GymEnv(cfg, sched, path, svc, sim_config_file=SAMPLE, test_mode=False)
    obs_ref, _ = env.reset(7)
    n = obs_ref.num_nodes
    lim = env.env_limits
    sim = load_batched_from_paths([path], svc, SAMPLE, cfg, num_envs=2)
    obs = sim.reset()
    np.testing.assert_allclose(obs[0, :n].numpy(), obs_ref.x.numpy(), rtol=1e-6, atol=1e-7)
    rng = np.random.default_rng(123)
    acts = random_actions(rng, steps, n, lim.MAX_SF_CHAIN_COUNT, lim.MAX_SERVICE_FUNCTION_COUNT)
    for k, a in enumerate(acts):
        o_ref, r_ref, _, _, _ = env.step(a.astype(np.float64))
        st = env.current_simulator_state.network_stats
        out = sim.step(torch.from_numpy(np.stack([a, a])))
        got = out.stats[0].numpy()
        assert (got[0], got[1]) == (st["run_successful_flows"], st["run_dropped_flows"]), f"step {k}"
        assert got[2] == env.simulator.metrics.metrics["run_generated_flows"], f"step {k}"
        assert abs(float(out.reward[0]) - r_ref) < 1e-5, f"step {k}"
        np.testing.assert_allclose(out.next_obs[0, :n].numpy(), o_ref.x.numpy(), rtol=1e-6, atol=1e-7)
        assert int(got[12]) == 0
        assert torch.equal(out.stats[0], out.stats[1])


def test_episode_reset_and_done():
    cfg = agent_cfg()
    cfg["episode_steps"] = 5
    sim = load_batched_from_paths([NETS["triangle"]], ABC, SAMPLE, cfg, num_envs=3)
    sim.reset()
    a = torch.zeros(3, sim.action_dim)
    am = sim.action_mask().view(24, 1, 3, 24)
    u = (am / 3.0).reshape(-1)
    a[:] = u
    dones, rets, run = [], [], torch.zeros(3, dtype=torch.float64)
    for _ in range(11):
        out = sim.step(a)
        dones.append(bool(out.done[0]))
        run += out.reward.double()
        if out.done[0]:
            # the finished episode's return is that episode's reward sum, not a running total
            assert torch.allclose(out.ep_return.double(), run, atol=1e-4), (out.ep_return, run)
            rets.append(run.clone())
            run.zero_()
    assert dones == [False] * 4 + [True] + [False] * 4 + [True] + [False]
    assert out.stats[0, 6] > 0
    assert len(rets) == 2


@pytest.mark.parametrize("simcfg", ["rand-arrival10_det-size001_duration100", "rand-mmp-arrival12-8_det-size001_dur100",
                                    "rand-arrival10_det-size001_duration100_trace_0_100_inall_chrate2_scale00005"])
def test_stochastic_configs_match_in_distribution(simcfg):
    """Poisson / MMPP / trace traffic: native Philox streams vs reference RNG streams agree in distribution."""
    cfg = agent_cfg()
    cfg["episode_steps"] = 100
    path = NETS["abilene"]
    p = cfg_path("config", "simulator", simcfg + ".yaml")
    env = GymEnv(cfg, {"training_network_files": [path], "inference_network": path, "period": 10}, path, ABC,
                 sim_config_file=p, test_mode=False)
    acts = random_actions(np.random.default_rng(0), 1, 11, 1, 3, density=1.0)
    a = acts[0]
    s = d = 0
    for seed in range(2):
        env.reset(seed)
        for _ in range(100):
            env.step(a.astype(np.float64))
            st = env.current_simulator_state.network_stats
            s += st["run_successful_flows"]
            d += st["run_dropped_flows"]
    E = 32
    sim = load_batched_from_paths([path], ABC, p, cfg, E)
    sim.reset()
    S = D = 0
    act = torch.from_numpy(np.tile(a, (E, 1)))
    for _ in range(100):
        out = sim.step(act)
        S += out.stats[:, 0].sum().item()
        D += out.stats[:, 1].sum().item()
    sim.check_flags()
    assert abs(S / (S + D) - s / (s + d)) < 0.02


@pytest.mark.parametrize("simcfg", ["sample_config", "rand-arrival10_det-size001_duration100",
                                    "rand-arrival10_det-size001_duration100_trace_0_100_inall_chrate2_scale00005",
                                    "rand-mmp-arrival12-8_det-size001_dur100", "pareto-size"])
def test_default_caps_headroom(simcfg, tmp_path):
    """Default pool capacities keep >= 2x headroom over the peaks of every shipped simulator config (and a
    Pareto-size config whose finish processes / link returns outlive their flows by seconds) under dense
    random schedules -- an overflow aborts a run (check_flags), so the margins must hold for bursty
    (MMPP, trace) as well as deterministic arrivals."""
    if simcfg == "pareto-size":
        c = yaml.safe_load(open(SAMPLE))
        c.update(deterministic_arrival=False, deterministic_size=False, flow_size_shape=2.5, flow_dr_stdev=0.2)
        p = tmp_path / "pareto.yaml"
        p.write_text(yaml.safe_dump(c))
        p = str(p)
    else:
        p = cfg_path("config", "simulator", simcfg + ".yaml")
    E = 8
    sim = load_batched_from_paths([NETS["abilene"]], ABC, p, agent_cfg(), E, device="cpu", seed=2, host_threads=4)
    sim.reset()
    rng = np.random.default_rng(0)
    mx = torch.zeros(16)
    for _ in range(60):
        o = sim.step(torch.from_numpy(rng.random((E, sim.action_dim), dtype=np.float32)))
        mx = torch.maximum(mx, o.stats.max(0).values)
    assert mx[12] == 0, f"flags {mx[12]}"
    d = sim.dims
    assert 2 * mx[13] <= d["event_cap"] and 2 * mx[14] <= d["proc_cap"] and 2 * mx[15] <= d["flow_cap"], (d, mx[13:])
