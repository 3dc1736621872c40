"""GPU: the exploration kernel's simulator hand-off (csrc/ops/explore.hip PMask) -- on 200-node topologies the
destination bitsets it writes from the post-processed rows drive the simulator exactly like the bitsets
sim_pmask_kernel derives from the stored action block (identical observations, rewards and stats)."""
import pytest
import torch
import yaml

from gsc_amd.ops.explore import explore_postprocess
from gsc_amd.sim.batched import load_batched_from_paths
from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu


def _sim(E, n_pad=None):
    nets = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(2)]
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "agent_syn200.yaml")))
    cfg["episode_steps"] = 4
    if n_pad is not None:
        cfg["max_nodes"] = n_pad
    return load_batched_from_paths(nets, cfg_path("service_functions", "abc-3sfc.yaml"),
                                   cfg_path("config", "simulator", "sample_config.yaml"), cfg, E, device="cuda",
                                   seed=11)


@pytest.mark.parametrize("n_pad", [None, 240], ids=["n_pad=N", "n_pad>N"])
def test_explore_pmask_handoff_matches_sim_pmask(n_pad):
    """n_pad > N: the simulator's bitset block holds the N = 200 source rows only; the exploration kernel must
    skip the action rows of sources 200..239 (they would otherwise overwrite the next env's state)."""
    E = 32
    runs = []
    for handoff in (True, False):
        sim = _sim(E, n_pad)
        assert sim.pmask_target() is not None, "200-node topologies use the HBM pmask bitsets"
        sim.set_topologies(torch.tensor([0, 1] * (E // 2)))
        sim.reset()
        from gsc_amd.models.graphs import GraphSet
        graphs = GraphSet(sim.topologies, sim.n_pad, sim.device)
        masks = graphs.action_masks(sim.C, sim.F)
        topo = sim.topo_cur.to(torch.int64).clone()
        g = torch.Generator(device="cuda").manual_seed(4)
        outs = []
        for step in range(6):
            mu = torch.rand(E, sim.action_dim, device="cuda", generator=g) * masks[topo]
            pm = sim.pmask_target() if handoff else None
            before = sim.states.clone() if pm is not None else None
            act = explore_postprocess(mu, masks, sim.n_pad, step < 2, 0.0, 0.3, seed=3, step=step, topo=topo,
                                      pmask=pm)
            if before is not None:   # only the bitset blocks change
                off = pm[0] - sim.states.data_ptr()
                rows = pm[6] * pm[4] * pm[5]
                keep = torch.ones(sim.state_bytes, dtype=torch.bool, device="cuda")
                keep[off:off + 32 * rows] = False
                assert off + 32 * rows <= sim.state_bytes
                assert torch.equal(sim.states[:, keep], before[:, keep])
            out = sim.step(act, buffer_set=step & 1, pmask_ready=handoff)
            outs.append(torch.cat([out.next_obs.flatten().float(), out.reward.float(), out.stats.flatten().float()]))
            topo = sim.topo_cur.to(torch.int64).clone()
        torch.cuda.synchronize()
        sim.check_flags()
        runs.append(torch.stack(outs))
    assert torch.equal(runs[0], runs[1])
