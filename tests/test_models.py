"""Model semantics: GATv2 (PyG formulas), embedder structure, mask folding, parameter counts."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F
import yaml

from gsc_amd.coordsim.reader import load_topology
from gsc_amd.models import Actor, GNNEmbedder, GraphSet, QNetwork, count_params
from tests.conftest import cfg_path

ABILENE = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
TRIANGLE = cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml")


def gatv2_literal(x, edge_index, p):
    """Per-message loop straight from PyG 2.3 GATv2Conv.forward/message + utils.softmax, aggr='mean'."""
    n = x.shape[0]
    xl = x @ p.lin_l_weight.T + p.lin_l_bias
    xr = x @ p.lin_r_weight.T + p.lin_r_bias
    ei = [(int(s), int(d)) for s, d in edge_index.T if s != d] + [(i, i) for i in range(n)]
    scores = [float((F.leaky_relu(xl[j] + xr[i], 0.2) * p.att[0]).sum()) for j, i in ei]
    out = torch.zeros(n, xl.shape[1], dtype=torch.float64)
    for i in range(n):
        ms = [k for k, (_, d) in enumerate(ei) if d == i]
        mx = max(scores[k] for k in ms)
        ex = {k: math.exp(scores[k] - mx) for k in ms}
        tot = sum(ex.values()) + 1e-16
        for k in ms:
            out[i] += (ex[k] / tot) * xl[ei[k][0]].double()
        out[i] /= len(ms)
    return out + p.bias.double()


def _cfg():
    return yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))


def test_param_counts_match_reference():
    cfg = _cfg()
    a, q = Actor(cfg, 3, 1728), QNetwork(cfg, 3, 1728)
    assert count_params(a) == 893628 and count_params(q) == 223997
    assert count_params(a.embedder) == 1276


def test_gatv2_dense_matches_literal_pyg_formulas():
    torch.manual_seed(0)
    topo = load_topology(ABILENE)
    gs = GraphSet([topo], 24)
    emb = GNNEmbedder(3, 22, 2, "mean", 2).double()
    x = torch.rand(1, 24, 3, dtype=torch.float64)
    x[:, topo.n:] = 0
    from gsc_amd.models.gnn import gatv2_dense_reference
    t = torch.zeros(1, dtype=torch.long)
    y = gatv2_dense_reference(x, gs.src[t], gs.dst[t], gs.valid[t], gs.deg[t].double(), emb.encoder)[0, :topo.n]
    ref = gatv2_literal(x[0, :topo.n], torch.from_numpy(topo.edge_index()), emb.encoder)
    torch.testing.assert_close(y, ref, rtol=1e-10, atol=1e-10)


def test_embedder_structure_and_pool():
    """encoder -> relu -> num_iter x shared process convs (relu between, none last) -> mean pool."""
    torch.manual_seed(1)
    topo = load_topology(ABILENE)
    gs = GraphSet([topo], 24)
    emb = GNNEmbedder(3, 22, 2, "mean", 2).double()
    x = torch.rand(2, 24, 3, dtype=torch.float64)
    x[:, topo.n:] = 0
    ei = torch.from_numpy(topo.edge_index())
    outs = []
    for b in range(2):
        h = torch.relu(gatv2_literal(x[b, :topo.n], ei, emb.encoder))
        h = torch.relu(gatv2_literal(h, ei, emb.process[0]))
        h = gatv2_literal(h, ei, emb.process[0])
        outs.append(h.mean(0))
    got = emb.forward_reference(x, torch.zeros(2, dtype=torch.long), gs)
    torch.testing.assert_close(got, torch.stack(outs), rtol=1e-9, atol=1e-9)


def test_native_embedder_rejects_unsupported_width():
    """GNN_features beyond every native kernel family fails up front with a clear error (not a kernel
    check at the first forward); the PyTorch reference still covers it."""
    topo = load_topology(ABILENE)
    gs = GraphSet([topo], 24)
    emb = GNNEmbedder(3, 80, 2, "mean", 2)
    x = torch.rand(2, 24, 3)
    tid = torch.zeros(2, dtype=torch.long)
    with pytest.raises(ValueError, match="GNN_features=80"):
        emb(x, tid, gs, use_native=True)
    assert emb(x, tid, gs, use_native=False).shape == (2, 80)


def test_mixed_topology_batch_is_per_graph():
    torch.manual_seed(2)
    topos = [load_topology(ABILENE), load_topology(TRIANGLE)]
    gs = GraphSet(topos, 24)
    emb = GNNEmbedder(3, 22, 2, "mean", 2)
    x = torch.rand(4, 24, 3)
    tid = torch.tensor([0, 1, 1, 0])
    x = x * gs.node_mask[tid].unsqueeze(-1)
    full = emb.forward_reference(x, tid, gs)
    for b in range(4):
        single = emb.forward_reference(x[b:b + 1], tid[b:b + 1], gs)
        torch.testing.assert_close(full[b:b + 1], single)


def test_mask_folding_equals_concatenation():
    torch.manual_seed(3)
    cfg = _cfg()
    topos = [load_topology(ABILENE), load_topology(TRIANGLE)]
    gs = GraphSet(topos, 24)
    masks = gs.action_masks(1, 3)
    q = QNetwork(cfg, 3, 1728).double()
    emb = torch.randn(5, 22, dtype=torch.float64)
    tid = torch.tensor([0, 1, 0, 1, 1])
    act = torch.rand(5, 1728, dtype=torch.float64)
    folded = q.mlp(emb, tid, masks.double(), act)
    full = q.mlp.forward_full(torch.cat([emb, masks.double()[tid], act], 1))
    torch.testing.assert_close(folded, full)
    a = Actor(cfg, 3, 1728).double()
    folded = a.mlp(emb, tid, masks.double())
    full = a.mlp.forward_full(torch.cat([emb, masks.double()[tid]], 1))
    torch.testing.assert_close(folded, full)


def test_composed_actor_critic_equals_materialised():
    """critic(x, actor(x)) via the re-associated action projection == the materialised path
    (values and gradients w.r.t. actor and critic parameters), one topology."""
    torch.manual_seed(0)
    cfg = _cfg()
    cfg["actor_hidden_layer_nodes"] = [32]
    cfg["critic_hidden_layer_nodes"] = [16]
    gs = GraphSet([load_topology(ABILENE)], 24, "cpu")
    masks = gs.action_masks(1, 3)
    actor, critic = Actor(cfg, 3, 1728), QNetwork(cfg, 3, 1728)
    x = torch.rand(6, 24, 3) * gs.node_mask[torch.zeros(6, dtype=torch.long)].unsqueeze(-1)
    topo = torch.zeros(6, dtype=torch.long)
    params = list(actor.parameters()) + list(critic.parameters())
    q1 = critic(x, topo, gs, masks, actor(x, topo, gs, masks))
    g1 = torch.autograd.grad(q1.sum(), params, allow_unused=True)
    q2 = critic.forward_on_actor(x, topo, gs, masks, actor, actor.hidden(x, topo, gs, masks))
    g2 = torch.autograd.grad(q2.sum(), params, allow_unused=True)
    torch.testing.assert_close(q1, q2, rtol=1e-5, atol=1e-5)
    for a, b in zip(g1, g2):
        if a is None:
            assert b is None or torch.count_nonzero(b) == 0
        else:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
