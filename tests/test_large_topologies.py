"""Large topologies (BASELINE configs 4/5): generated 50-node + trace + 3 SFCs and 200-node
scheduler-driven configs run through the batched simulator and the trainer (CPU host path)."""
import numpy as np
import pytest
import torch
import yaml

from gsc_amd.coordsim.reader import load_topology
from gsc_amd.models import GNNEmbedder, GraphSet
from gsc_amd.sim.batched import load_batched_from_paths
from tests.conftest import cfg_path

SYN50 = cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml")
SYN200 = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(4)]
SVC3 = cfg_path("service_functions", "abc-3sfc.yaml")


def _cfg(name):
    return yaml.safe_load(open(cfg_path("config", "agent", name + ".yaml")))


def test_generator_properties(tmp_path):
    import networkx as nx
    from scripts.gen_networks import make_trace, synthetic_topology
    g = synthetic_topology(60, 5, degree=3, seed=9)
    assert nx.is_connected(g) and g.number_of_nodes() == 60
    assert sum(d["NodeType"] == "Ingress" for _, d in g.nodes(data=True)) == 5
    f = tmp_path / "g.graphml"
    nx.write_graphml(g, f)
    t = load_topology(str(f))
    assert t.n == 60 and len(t.ingress) == 5 and t.diameter > 0
    tr = make_trace(str(f), str(tmp_path / "t.csv"), duration_ms=1000, interval_ms=200)
    rows = open(tr).read().splitlines()
    assert rows[0] == "time,node,inter_arrival_mean" and len(rows) == 1 + 5 * 5


def test_syn50_trainer_steps():
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    cfg = _cfg("agent_syn50")
    cfg["actor_hidden_layer_nodes"] = [32]
    sim = load_batched_from_paths([SYN50], SVC3, cfg_path("config", "simulator", "rand-arrival12_trace_syn50.yaml"),
                                  cfg, 4, device="cpu", seed=1)
    assert sim.action_dim == 50 * 3 * 3 * 50
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=4, batch_size=8, learning_starts=2, check_every=0))
    for _ in range(4):
        tr.step()
    m = tr.metrics()
    assert tr.learner.updates == 3 and m["succ"] + m["drop"] > 0 and np.isfinite(m["qf1_loss"])


def test_syn200_sim_and_scheduler():
    cfg = _cfg("agent_syn200")
    cfg["episode_steps"] = 3
    sim = load_batched_from_paths(SYN200, SVC3, cfg_path("config", "simulator", "sample_config.yaml"), cfg, 4,
                                  device="cpu", seed=2)
    sim.set_topologies([0, 1, 2, 3])
    sim.reset()
    assert torch.equal(sim.topo_cur.long(), torch.arange(4))
    a = torch.zeros(4, sim.action_dim)
    for e in range(4):
        a[e] = sim.action_mask(e) / sim.topologies[e].n
    sim.set_topologies(1)       # next episode: every env moves to topology 1
    for _ in range(3):
        out = sim.step(a)
    assert bool(out.done.all()) and torch.equal(sim.topo_cur.long(), torch.ones(4, dtype=torch.long))
    assert float(out.stats[:, 6].sum()) > 0
    sim.check_flags()


def test_gnn_native_path_for_graphs_beyond_lds():
    """50-node graphs run the two-tile fused kernels, 200-node graphs the large-graph fused kernels (gnn_lg.hip:
    one graph per workgroup, all convs in LDS) at GSC's width; shapes beyond their LDS budget (H = 32 at 200
    nodes) run the layer-wise native kernels (gsc_amd/ops/gnn_lw.py) -- no PyTorch GNN on the GPU (GPU numerics:
    tests/test_gpu_gnn_lg.py, tests/test_gpu_gnn_lw.py)."""
    import inspect
    from gsc_amd.models import gnn as gnn_mod
    from gsc_amd.ops.gnn import gnn_fits
    e = GNNEmbedder(3, 22, 2, "mean", 2)
    assert gnn_fits(e, GraphSet([load_topology(SYN50)], 50, "cpu"), 50, 3)
    assert gnn_fits(e, GraphSet([load_topology(SYN200[0])], 200, "cpu"), 200, 3)
    assert not gnn_fits(GNNEmbedder(3, 32, 2, "mean", 2), GraphSet([load_topology(SYN200[0])], 200, "cpu"), 200, 3)
    assert not gnn_fits(GNNEmbedder(3, 22, 3, "mean", 1), GraphSet([load_topology(SYN200[0])], 200, "cpu"), 200, 3)
    src = inspect.getsource(gnn_mod.GNNEmbedder.forward)
    assert "gnn_embed_layerwise" in src
