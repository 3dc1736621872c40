"""Golden fixed-policy outcomes of the reference simulator (SURVEY.md section 4 / BASELINE.md)."""
import numpy as np
import pytest
import yaml

from gsc_amd.coordsim import Simulator
from gsc_amd.envs import ActionScheduleProcessor, GymEnv
from gsc_amd.spinterface import SimulatorAction
from tests.conftest import cfg_path

ABILENE = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
TRIANGLE = cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml")
ABC = cfg_path("service_functions", "abc.yaml")
SAMPLE = cfg_path("config", "simulator", "sample_config.yaml")


def _uniform_action(sim_state):
    nodes = [n["id"] for n in sim_state.network["nodes"]]
    sfs = ["a", "b", "c"]
    sched = {v: {"sfc_1": {sf: {w: 1 / len(nodes) for w in nodes} for sf in sfs}} for v in nodes}
    return SimulatorAction({v: set(sfs) for v in nodes}, sched)


def test_first_windows_direct_apply():
    sim = Simulator(ABILENE, ABC, SAMPLE)
    st = sim.init(1234)
    act = _uniform_action(st)
    got = []
    for _ in range(3):
        st = sim.apply(act)
        got.append((sim.metrics.metrics["run_generated_flows"], st.network_stats["run_successful_flows"],
                    st.network_stats["run_dropped_flows"]))
    assert got == [(36, 10, 24), (40, 13, 27), (40, 12, 28)]


def _env(network):
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    sched = {"training_network_files": [network], "inference_network": network, "period": 10}
    return GymEnv(cfg, sched, network, ABC, sim_config_file=SAMPLE, test_mode=False)


def _run(env, policy, seed, steps=200):
    lim = env.env_limits
    proc = ActionScheduleProcessor(lim.MAX_NODE_COUNT, lim.MAX_SF_CHAIN_COUNT, lim.MAX_SERVICE_FUNCTION_COUNT)
    obs, _ = env.reset(seed)
    n = obs.num_nodes
    succ = drop = 0
    rewards = []
    for _ in range(steps):
        a = np.zeros(lim.scheduling_shape)
        if policy == "uniform":
            a[:n, :, :, :n] = 1 / n
        else:
            for i in range(n):
                a[i, :, :, i] = 1
        obs, r, done, _, _ = env.step(proc.process_action(a.reshape(-1)))
        s = env.current_simulator_state.network_stats
        succ += s["run_successful_flows"]
        drop += s["run_dropped_flows"]
        rewards.append(r)
    return succ, drop, float(np.mean(rewards)), done


@pytest.mark.parametrize("seed", [1, 999])
def test_abilene_uniform_golden(seed):
    succ, drop, mean_r, done = _run(_env(ABILENE), "uniform", seed)
    assert (succ, drop) == (2798, 5196)
    assert abs(mean_r - (-0.300)) < 1e-3
    assert done


def test_abilene_local_zero_success():
    succ, drop, _, _ = _run(_env(ABILENE), "local", 1234)
    assert succ == 0 and drop > 7900


def test_triangle_uniform_full_success():
    succ, drop, _, _ = _run(_env(TRIANGLE), "uniform", 1234)
    assert (succ, drop) == (1997, 0)
