"""GPU: layer-wise GATv2 kernels (node linears, per-graph / per-node attention kernels, one-pass conv
gradients) vs the fp32 PyTorch reference -- the native path for graphs beyond one CU's LDS (200-node syn topologies,
BASELINE config 5); also exercised on 50-node and Abilene graphs by calling it directly."""
import pytest
import torch

from gsc_amd.coordsim.reader import load_topology
from gsc_amd.models import GNNEmbedder, GraphSet
from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu
DEV = "cuda"
SYN200 = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(3)]


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _check(gs, P, B, layers=2, iters=2, hidden=22, direct=False):
    from gsc_amd.ops.gnn import gnn_embed_layerwise
    torch.manual_seed(0)
    emb = GNNEmbedder(3, hidden, layers, "mean", iters).to(DEV)
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV)
    x = torch.rand(B, P, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    params = list(emb.parameters())
    ref = emb.forward_reference(x, topo, gs)
    w = torch.linspace(-1, 1, hidden, device=DEV)
    gref = torch.autograd.grad((ref * w).sum(), params)
    out = gnn_embed_layerwise(emb, x, topo, gs) if direct else emb(x, topo, gs, use_native=True)
    gout = torch.autograd.grad((out * w).sum(), params)
    # bf16 GEMM operands (node linears, dW, dX W); everything else fp32
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    for i, (a, b) in enumerate(zip(gout, gref)):
        assert _rel(a, b) < 3e-2, (i, a.shape, _rel(a, b))
    return out


def test_layerwise_200_nodes_is_the_native_path_without_lg(monkeypatch):
    """GSC_GNN_LG=0 routes 200-node graphs back to the layer-wise kernels (the large-graph fused kernels'
    A/B partner)."""
    from gsc_amd.ops.gnn import gnn_fits
    monkeypatch.setenv("GSC_GNN_LG", "0")
    gs = GraphSet([load_topology(p) for p in SYN200], 200, DEV)
    emb = GNNEmbedder(3, 22, 2, "mean", 2)
    assert not gnn_fits(emb, gs, 200, 3)
    _check(gs, 200, 96)


@pytest.mark.parametrize("case", ["syn50", "abilene-bteurope"])
def test_layerwise_matches_reference_small_graphs(case):
    if case == "syn50":
        gs = GraphSet([load_topology(cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml"))], 50, DEV)
        P = 50
    else:
        gs = GraphSet([load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")),
                       load_topology(cfg_path("networks", "bteurope", "bteurope-in4-rand-cap0-2.graphml"))], 24, DEV)
        P = 24
    _check(gs, P, 300, direct=True)


@pytest.mark.parametrize("layers,iters,hidden", [(1, 1, 22), (3, 1, 16), (2, 2, 32), (2, 1, 8)])
def test_layerwise_shapes(layers, iters, hidden):
    """hidden 22 / 32: the staged MFMA kernels; 16 with a next conv (its fused linears' MFMA image does not
    fit at n_pad 200) and 8: the lane-per-node kernels."""
    gs = GraphSet([load_topology(p) for p in SYN200[:2]], 200, DEV)
    _check(gs, 200, 40, layers, iters, hidden, direct=True)


def test_native_update_uses_layerwise_for_200_nodes(monkeypatch):
    """With GSC_GNN_LG=0 the native DDPG update runs the layer-wise embedder (no PyTorch GNN) on 200-node graphs."""
    import yaml
    monkeypatch.setenv("GSC_GNN_LG", "0")
    from gsc_amd.agents import Batch, DDPGLearner
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "agent_syn200.yaml")))
    gs = GraphSet([load_topology(p) for p in SYN200], 200, DEV)
    C, F = 3, 3
    A = 200 * C * F * 200
    L = DDPGLearner(cfg, 3, A, gs, C, F, DEV, seed=1)
    assert L.native_ok
    B = 64
    g = torch.Generator(device=DEV).manual_seed(0)
    topo = torch.randint(0, 3, (B,), device=DEV, generator=g)
    obs = torch.rand(B, 200, 3, device=DEV, generator=g) * gs.node_mask[topo].unsqueeze(-1)
    nxt = torch.rand(B, 200, 3, device=DEV, generator=g) * gs.node_mask[topo].unsqueeze(-1)
    b = Batch(obs, topo, torch.rand(B, A, device=DEV, generator=g).to(torch.bfloat16),
              torch.rand(B, device=DEV, generator=g), nxt, torch.zeros(B, device=DEV))
    before = L.actor_flat.flat.clone()
    for _ in range(2):
        L.update(b)
    torch.cuda.synchronize()
    assert L._native is not None and L._native.layerwise
    assert torch.isfinite(L.actor_flat.flat).all() and not torch.equal(before, L.actor_flat.flat)
    assert all(float(v) == float(v) for v in L.last.values())


@pytest.mark.parametrize("hidden", [40, 64])
def test_layerwise_wide_hidden(hidden):
    """More than 32 channels: one whole wave per node (lw_*_kernel<64>), Abilene + BtEurope."""
    gs = GraphSet([load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")),
                   load_topology(cfg_path("networks", "bteurope", "bteurope-in4-rand-cap0-2.graphml"))], 24, DEV)
    _check(gs, 24, 333, hidden=hidden, direct=True)


def test_layerwise_200_nodes_wide_hidden_per_node_kernel():
    """200 nodes x 64 channels: the graph's x_l / x_r block (100 KB) exceeds the per-graph kernel's LDS
    budget, so the forward takes the per-node attention kernel."""
    gs = GraphSet([load_topology(p) for p in SYN200[:2]], 200, DEV)
    _check(gs, 200, 24, hidden=64, direct=True)


@pytest.mark.parametrize("layers,iters,hidden", [(2, 2, 22), (1, 1, 22), (3, 1, 16), (2, 2, 32)])
def test_layerwise_forward_without_backward(layers, iters, hidden):
    """No-grad forwards (target / act embedders): the per-conv kernels without stored rows / alpha; same
    tolerance as the saved path."""
    from gsc_amd.ops.gnn import gnn_embed_layerwise
    gs = GraphSet([load_topology(p) for p in SYN200], 200, DEV)
    torch.manual_seed(1)
    emb = GNNEmbedder(3, hidden, layers, "mean", iters).to(DEV)
    B = 64
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV)
    x = torch.rand(B, 200, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    with torch.no_grad():
        ref = emb.forward_reference(x, topo, gs)
        out = gnn_embed_layerwise(emb, x, topo, gs)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
