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
