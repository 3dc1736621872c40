"""GPU: the HIP simulator kernel must match the host path of the same C++ core bit-for-bit."""
import numpy as np
import pytest
import torch
import yaml

from gsc_amd.sim.batched import load_batched_from_paths
from tests.conftest import cfg_path
from tests.test_batched_sim_diff import random_actions

pytestmark = pytest.mark.gpu

ABC = cfg_path("service_functions", "abc.yaml")
NET = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")


def _cfg():
    c = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    c["episode_steps"] = 20
    return c


@pytest.mark.parametrize("simcfg", ["sample_config", "rand-arrival10_det-size001_duration100",
                                    "rand-mmp-arrival12-8_det-size001_dur100"])
def test_device_matches_host(simcfg):
    assert torch.cuda.is_available()
    p = cfg_path("config", "simulator", simcfg + ".yaml")
    E = 96
    host = load_batched_from_paths([NET], ABC, p, _cfg(), E, device="cpu", seed=3)
    dev = load_batched_from_paths([NET], ABC, p, _cfg(), E, device="cuda", seed=3)
    o_h = host.reset().clone()
    o_d = dev.reset().cpu()
    assert torch.equal(o_h, o_d)
    acts = random_actions(np.random.default_rng(1), 45, 11, 1, 3)
    for k, a in enumerate(acts):
        A = torch.from_numpy(np.tile(a, (E, 1)))
        oh = host.step(A)
        od = dev.step(A.cuda())
        torch.cuda.synchronize()
        assert torch.equal(oh.stats, od.stats.cpu()), f"step {k}"
        assert torch.equal(oh.obs, od.obs.cpu()), f"step {k}"
        assert torch.equal(oh.reward, od.reward.cpu())
        assert torch.equal(oh.done, od.done.cpu())
    dev.check_flags()


SYN50 = cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml")
SYN200 = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(4)]
SVC3 = cfg_path("service_functions", "abc-3sfc.yaml")


@pytest.mark.parametrize("case", ["syn50-trace", "syn200"])
def test_device_matches_host_large(case):
    """50-node (3 SFCs + trace; topology tables staged in LDS) and 200-node (tables in HBM) topologies."""
    if case == "syn50-trace":
        nets, simcfg, agent = [SYN50], cfg_path("config", "simulator", "rand-arrival12_trace_syn50.yaml"), "agent_syn50"
    else:
        nets, simcfg, agent = SYN200, cfg_path("config", "simulator", "sample_config.yaml"), "agent_syn200"
    cfg = yaml.safe_load(open(cfg_path("config", "agent", agent + ".yaml")))
    cfg["episode_steps"] = 6
    E = 16
    host = load_batched_from_paths(nets, SVC3, simcfg, cfg, E, device="cpu", seed=5, topo_init=np.arange(E) % len(nets))
    dev = load_batched_from_paths(nets, SVC3, simcfg, cfg, E, device="cuda", seed=5, topo_init=np.arange(E) % len(nets))
    assert torch.equal(host.reset().clone(), dev.reset().cpu())
    rng = np.random.default_rng(2)
    for k in range(8):
        a = torch.from_numpy(rng.random((E, host.action_dim), dtype=np.float32))
        oh, od = host.step(a), dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(oh.stats, od.stats.cpu()), f"step {k}"
        assert torch.equal(oh.obs, od.obs.cpu()), f"step {k}"
    dev.check_flags()


def test_device_matches_host_syn200_256_envs():
    """256 envs of 200-node topologies (one rank's share of a 2,048-env 8-GPU job): device == host over an
    episode end (topology switch at the reset), with the heavy uniform schedule of scripts/sim_throughput.py
    (every node forwards to every node: long paths, many pending link returns) and the cycle-counting
    variant enabled for the second half (it must not touch memory outside its counters)."""
    from gsc_amd.envs import threshold_normalize
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "agent_syn200.yaml")))
    cfg["episode_steps"] = 4
    E = 256
    simcfg = cfg_path("config", "simulator", "sample_config.yaml")
    nets = SYN200[:3]
    host = load_batched_from_paths(nets, SVC3, simcfg, cfg, E, device="cpu", seed=7, topo_init=np.arange(E) % 3)
    dev = load_batched_from_paths(nets, SVC3, simcfg, cfg, E, device="cuda", seed=7, topo_init=np.arange(E) % 3)
    nxt = (np.arange(E) + 1) % 3
    host.set_topologies(nxt)
    dev.set_topologies(nxt)
    assert torch.equal(host.reset().clone(), dev.reset().cpu())
    P, n = host.n_pad, host.topologies[0].n
    rng = np.random.default_rng(4)
    a = np.zeros((P, host.C, host.F, P))
    a[:n, :, :, :n] = rng.random((n, host.C, host.F, n))
    uni = threshold_normalize(a.reshape(-1), P, 0.1, 2).astype(np.float32)
    for k in range(7):
        if k == 3:
            dev.enable_profiling()
        a = np.tile(uni, (E, 1)) if k % 2 == 0 else rng.random((E, host.action_dim), dtype=np.float32)
        a = torch.from_numpy(a)
        oh, od = host.step(a), dev.step(a.cuda())
        torch.cuda.synchronize()
        assert torch.equal(oh.stats, od.stats.cpu()), f"step {k}"
        assert torch.equal(oh.obs, od.obs.cpu()), f"step {k}"
        assert torch.equal(oh.reward, od.reward.cpu()), f"step {k}"
    assert int(dev.prof[E * 4:].view(E, 64, 2)[:, :, 1].sum()) > 0
    dev.check_flags()
    host.check_flags()
