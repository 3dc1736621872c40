"""GPU: the large-graph fused GATv2 kernels (csrc/ops/gnn_lg.hip: one 200-node graph per workgroup, every conv in
LDS, recomputing backward) vs the fp32 PyTorch reference (gsc_amd/models/gnn.py::gatv2_dense_reference, the
reference's PyG GATv2Conv semantics, src/rlsp/agents/models.py:10-53).  bf16 MFMA operands (node linears, dW,
dX W) and bf16 inter-conv images, everything else fp32: the same tolerances as the other MFMA families."""
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


def _mixed(P=200):
    """200-node topologies next to a 50-node and an 11-node one (padded rows, idle lane pairs) in one batch."""
    topos = [load_topology(p) for p in SYN200] + [
        load_topology(cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml")),
        load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))]
    return GraphSet(topos, P, DEV)


def _check(gs, P, B, layers=2, iters=2, hidden=22, seed=0, tol=3e-2):
    from gsc_amd.native import load
    from gsc_amd.ops.gnn import _tables, gnn_fits
    torch.manual_seed(seed)
    emb = GNNEmbedder(3, hidden, layers, "mean", iters).to(DEV)
    assert gnn_fits(emb, gs, P, 3), "expected the large-graph fused kernels"
    assert load().gnn_saved_bytes(_tables(gs), P, 3, hidden, [0] + [1] * (iters * (layers - 1))) == 0
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV)
    x = torch.rand(B, P, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    params = list(emb.parameters())
    ref = emb.forward_reference(x, topo, gs)
    w = torch.linspace(-1, 1, hidden, device=DEV)
    gref = torch.autograd.grad((ref * w).sum(), params)
    out = emb(x, topo, gs, use_native=True)
    gout = torch.autograd.grad((out * w).sum(), params)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    for i, (a, b) in enumerate(zip(gout, gref)):
        assert _rel(a, b) < tol, (i, a.shape, _rel(a, b))
    return emb, x, topo, out, gout


@pytest.mark.parametrize("hidden", [22, 16, 23, 12])
def test_lg_matches_reference_syn200(hidden):
    gs = GraphSet([load_topology(p) for p in SYN200], 200, DEV)
    _check(gs, 200, 300, hidden=hidden)


def test_lg_two_convs():
    """L = 2: the input image and conv 0's saved output share the one slot."""
    gs = GraphSet([load_topology(p) for p in SYN200[:2]], 200, DEV)
    _check(gs, 200, 64, iters=1)


def test_lg_mixed_sizes_and_padding():
    """200 / 50 / 11-node graphs at n_pad 200 and at n_pad 208 (padded rows and node groups)."""
    _check(_mixed(200), 200, 250)
    _check(_mixed(208), 208, 97, seed=1)


def test_lg_deterministic_and_forward2():
    """Bitwise reproducible gradients (per-workgroup rows, fixed-order sums); gnn_forward2 == two forwards."""
    from gsc_amd.native import load
    from gsc_amd.ops.gnn import _flat, _layer_of, _tables
    gs = _mixed(200)
    torch.manual_seed(3)
    emb = GNNEmbedder(3, 22, 2, "mean", 2).to(DEV)
    B = 1000
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV)
    x = torch.rand(B, 200, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    runs = []
    for _ in range(2):
        out = emb(x, topo, gs, use_native=True)
        runs.append(torch.autograd.grad(out.square().sum(), list(emb.parameters())))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    nat = load()
    e2 = GNNEmbedder(3, 22, 2, "mean", 2).to(DEV)
    p1, p2 = _flat(emb.flat_parameters()).contiguous(), _flat(e2.flat_parameters()).contiguous()
    t32 = topo.to(torch.int32)
    s = torch.cuda.current_stream().cuda_stream
    ref = [torch.empty(B, 22, device=DEV) for _ in range(2)]
    for p, o in zip((p1, p2), ref):
        nat.gnn_forward(_tables(gs), p.data_ptr(), x.data_ptr(), t32.data_ptr(), o.data_ptr(), B, 200, 3, 22,
                        _layer_of(emb), s, 0)
    got = [torch.empty(B, 22, device=DEV) for _ in range(2)]
    nat.gnn_forward2(_tables(gs), p1.data_ptr(), p2.data_ptr(), x.data_ptr(), t32.data_ptr(), got[0].data_ptr(),
                     got[1].data_ptr(), B, 200, 3, 22, _layer_of(emb), s)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_lg_cu_budget_grid():
    """A CU budget (the trainer's masked learner stream) switches both kernels to the full-device grid claiming
    graphs from a zeroed work-queue counter (csrc/ops/gnn.hip::work_slot); same numerics."""
    from gsc_amd.native import load
    nat = load()
    nat.gnn_set_cu_budget(48)
    try:
        _check(GraphSet([load_topology(p) for p in SYN200], 200, DEV), 200, 500)
    finally:
        nat.gnn_set_cu_budget(0)


SYN50 = [cfg_path("networks", "synthetic", f"syn50-in8-cap1-3{s}.graphml") for s in ("", "-s1", "-s2", "-s3")]


@pytest.mark.parametrize("hidden", [22, 16])
def test_lg_packs_of_50_node_graphs(hidden):
    """BASELINE config-4 shape (n_pad 50): five graphs per workgroup as one disjoint 250-node graph; B = 1,003 leaves
    a partial last pack (its missing graphs are empty)."""
    gs = GraphSet([load_topology(p) for p in SYN50], 50, DEV)
    _check(gs, 50, 1003, hidden=hidden)


def test_lg_packs_mixed_sizes():
    """n_pad 64 (packs of four): 50 / 53 / 42 / 11-node graphs, padded rows and padded graphs in one pack."""
    topos = [load_topology(SYN50[0]), load_topology(cfg_path("networks", "tinet", "tinet-in4-rand-cap0-2.graphml")),
             load_topology(cfg_path("networks", "chinanet", "chinanet-in4-rand-cap0-2.graphml")),
             load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))]
    _check(GraphSet(topos, 64, DEV), 64, 777, seed=2)
