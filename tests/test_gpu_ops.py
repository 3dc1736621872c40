"""GPU numerics: HIP kernels vs PyTorch fp32 references."""
import numpy as np
import pytest
import torch
import yaml

from gsc_amd.coordsim.reader import load_topology
from gsc_amd.models import GNNEmbedder, GraphSet
from gsc_amd.ops import FlatParams, FusedAdamPolyak, adam_polyak_reference, explore_postprocess, \
    normalize_slices_reference
from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graphs(dev):
    topos = [load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")),
             load_topology(cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml")),
             load_topology(cfg_path("networks", "bteurope", "bteurope-in4-rand-cap0-2.graphml"))]
    return GraphSet(topos, 24, dev)


def _mid_graphs(dev, P=64):
    """33..64-node topologies (two 32-node MFMA tiles: gnn_mt.hip) next to an 11-node one."""
    topos = [load_topology(cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml")),
             load_topology(cfg_path("networks", "tinet", "tinet-in4-rand-cap0-2.graphml")),
             load_topology(cfg_path("networks", "chinanet", "chinanet-in4-rand-cap0-2.graphml")),
             load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))]
    return GraphSet(topos, P, dev)


@pytest.mark.parametrize("layers,iters,hidden,fused", [(2, 2, 22, True), (2, 2, 16, True), (2, 2, 32, True),
                                                       (2, 3, 22, True), (1, 1, 22, False), (3, 1, 22, False),
                                                       (2, 2, 40, False)])
def test_gnn_native_matches_reference(layers, iters, hidden, fused):
    """Native embedder vs the fp32 PyTorch reference on Abilene (11 nodes), triangle and BtEurope (24
    nodes) in one batch.  GSC shapes (encoder + one shared process block, H <= 32) run the MFMA
    kernels of gnn_mf.hip; the others run the layer-wise kernels (gnn_lw.py).  bf16 operands."""
    from gsc_amd.ops.gnn import gnn_use_fused
    gs = _graphs(DEV)
    assert gnn_use_fused(GNNEmbedder(3, hidden, layers, "mean", iters), gs, 24, 3) == fused
    _check_gnn(layers, iters, hidden, gs, bf16=True)


@pytest.mark.parametrize("pack", ["1", "0"], ids=["lg-pack", "mt"])
@pytest.mark.parametrize("hidden", [22, 32, 16])
def test_gnn_mfma_two_tiles_matches_reference(hidden, pack, monkeypatch):
    """33..64-node graphs: 50-node synthetic, TiNet (53), ChinaNet (42) and Abilene (11, second tile empty) in one
    batch, forward + backward vs fp32 -- on the two-tile MFMA kernels (gnn_mt.hip; GSC_GNN_LG_PACK=0, and H = 32
    always) and in packs of four graphs on the large-graph kernels (gnn_lg.hip, H <= 31: nothing saved)."""
    from gsc_amd.native import load
    from gsc_amd.ops.gnn import _tables, gnn_use_fused
    monkeypatch.setenv("GSC_GNN_LG_PACK", pack)
    gs = _mid_graphs(DEV)
    emb = GNNEmbedder(3, hidden, 2, "mean", 2)
    assert gnn_use_fused(emb, gs, 64, 3)
    saved = load().gnn_saved_bytes(_tables(gs), 64, 3, hidden, [0, 1, 1])
    assert (saved == 0) == (pack == "1" and hidden <= 31), saved
    _check_gnn(2, 2, hidden, gs, 64, bf16=True)


def test_gnn_50_nodes_padded_50():
    """BASELINE config-4 shape: n_pad = 50 (the agent's max_nodes), 50-node topology + Abilene."""
    gs = GraphSet([load_topology(cfg_path("networks", "synthetic", "syn50-in8-cap1-3.graphml")),
                   load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))], 50, DEV)
    _check_gnn(2, 2, 22, gs, 50, bf16=True)


@pytest.mark.parametrize("pack", ["1", "0"], ids=["lg-pack", "mt"])
def test_gnn_mfma_two_tiles_work_queue(pack, monkeypatch):
    """The overlap mode's two-tile backward: a CU budget set (as the trainer does for its masked learner
    stream) switches the backward to a full-device grid claiming graphs (gnn_mt) or packs (gnn_lg) from a zeroed
    counter; the gradients must match the fp32 reference as with the fixed-stride grid."""
    from gsc_amd.native import load
    monkeypatch.setenv("GSC_GNN_LG_PACK", pack)
    nat = load()
    nat.gnn_set_cu_budget(64)
    try:
        _check_gnn(2, 2, 22, _mid_graphs(DEV), 64, bf16=True)
    finally:
        nat.gnn_set_cu_budget(0)


@pytest.mark.parametrize("mid", [False, True], ids=["one-tile", "two-tile"])
def test_gnn_forward_two_parameter_sets(mid):
    """gnn_forward2 (target actor + target critic embedders in one launch) == two gnn_forward launches."""
    from gsc_amd.native import load
    from gsc_amd.ops.gnn import _flat, _layer_of, _tables
    nat = load()
    torch.manual_seed(4)
    gs = _mid_graphs(DEV) if mid else _graphs(DEV)
    P = 64 if mid else 24
    e1, e2 = GNNEmbedder(3, 22, 2, "mean", 2).to(DEV), GNNEmbedder(3, 22, 2, "mean", 2).to(DEV)
    p1, p2 = _flat(e1.flat_parameters()).contiguous(), _flat(e2.flat_parameters()).contiguous()
    B = 1000
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV, dtype=torch.int32)
    x = torch.rand(B, P, 3, device=DEV) * gs.node_mask[topo.long()].unsqueeze(-1)
    s = torch.cuda.current_stream().cuda_stream
    ref = [torch.empty(B, 22, device=DEV) for _ in range(2)]
    for p, o in zip((p1, p2), ref):
        nat.gnn_forward(_tables(gs), p.data_ptr(), x.data_ptr(), topo.data_ptr(), o.data_ptr(), B, P, 3, 22,
                        _layer_of(e1), s, 0)
    got = [torch.empty(B, 22, device=DEV) for _ in range(2)]
    nat.gnn_forward2(_tables(gs), p1.data_ptr(), p2.data_ptr(), x.data_ptr(), topo.data_ptr(), got[0].data_ptr(),
                     got[1].data_ptr(), B, P, 3, 22, _layer_of(e1), s)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mid", [False, True], ids=["one-tile", "two-tile"])
def test_gnn_mfma_deterministic(mid):
    """MFMA gradients are bitwise reproducible (per-workgroup partial rows, fixed-order sums)."""
    torch.manual_seed(3)
    gs = _mid_graphs(DEV) if mid else _graphs(DEV)
    P = 64 if mid else 24
    emb = GNNEmbedder(3, 22, 2, "mean", 2).to(DEV)
    topo = torch.randint(0, gs.num_topologies, (4096,), device=DEV)
    x = torch.rand(4096, P, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    runs = []
    for _ in range(2):
        out = emb(x, topo, gs, use_native=True)
        runs.append(torch.autograd.grad(out.square().sum(), list(emb.parameters())))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def _check_gnn(layers, iters, hidden, gs=None, P=24, bf16=False):
    torch.manual_seed(0)
    gs = gs if gs is not None else _graphs(DEV)
    emb = GNNEmbedder(3, hidden, layers, "mean", iters).to(DEV)
    B = 777
    topo = torch.randint(0, gs.num_topologies, (B,), device=DEV)
    x = torch.rand(B, P, 3, device=DEV) * gs.node_mask[topo].unsqueeze(-1)
    params = list(emb.parameters())
    ref = emb.forward_reference(x, topo, gs)
    w = torch.linspace(-1, 1, hidden, device=DEV)
    gref = torch.autograd.grad((ref * w).sum(), params)
    out = emb(x, topo, gs, use_native=True)
    gout = torch.autograd.grad((out * w).sum(), params)
    if bf16:
        def rel(a, b):
            return float((a - b).norm() / b.norm().clamp_min(1e-12))
        assert rel(out, ref) < 1e-2, rel(out, ref)
        for i, (a, b) in enumerate(zip(gout, gref)):
            assert rel(a, b) < 2e-2, (i, a.shape, rel(a, b))
        return
    torch.testing.assert_close(out, ref, rtol=2e-5, atol=2e-5)
    for a, b in zip(gout, gref):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3)


def test_adam_polyak_matches_reference():
    torch.manual_seed(1)
    n = 100003
    p = torch.randn(n, device=DEV)
    tgt = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    p2, t2, m2, v2 = p.clone(), tgt.clone(), m.clone(), v.clone()
    lin = torch.nn.Linear(1, 1).to(DEV)
    fp = FlatParams(lin)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV)
        adam_polyak_reference(p2, g, m2, v2, t2, step, 1e-3, (0.9, 0.999), 1e-8, 1e-2)
        fp.flat = p
        fp.grad = g
        opt = FusedAdamPolyak.__new__(FusedAdamPolyak)
        opt.fp, opt.lr, opt.betas, opt.eps, opt.wd, opt.tau = fp, 1e-3, (0.9, 0.999), 1e-8, 0.0, 1e-2
        opt.target = type("T", (), {"flat": tgt})()
        opt.m, opt.v = m, v
        opt.step_t = torch.full((), step - 1, dtype=torch.int64, device=DEV)  # device step counter
        opt._host_step = step - 1
        opt.guard, opt.guard_enabled = torch.zeros(4, dtype=torch.int32, device=DEV), True
        opt.step()
        assert opt.step_count == step
    torch.testing.assert_close(p, p2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(tgt, t2, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("P,n", [(24, 11), (50, 50), (64, 37), (200, 200), (200, 131), (199, 150), (225, 200)])
def test_explore_postprocess_device(P, n):
    """Lane-parallel kernels: two slices per wave (n_pad <= 32), one slice per wave with 1-4 weights per
    lane (n_pad <= 256, the 50- and 200-node configs)."""
    torch.manual_seed(2)
    E = 64 if P <= 64 else 8
    A = P * 3 * P
    mask = torch.zeros(E, P, 3, P, device=DEV)
    mask[:, :n, :, :n] = 1
    mask = mask.view(E, A)
    mu = torch.rand(E, A, device=DEV) * mask
    for warm in (True, False):
        out = explore_postprocess(mu, mask, P, warm, 0.0, 0.3, seed=5, step=7)
        s = out.view(E, -1, P).double().sum(-1)
        assert torch.allclose(s, torch.ones_like(s), atol=1e-6)
        # idempotent under the reference post-processing (already thresholded + normalised)
        again = normalize_slices_reference(out.view(E, -1, P).cpu().double(), 0.1, 2).float().view(E, A)
        torch.testing.assert_close(out.cpu(), again, rtol=1e-6, atol=1e-6)
    # noise-free path equals the reference exactly
    out = explore_postprocess(mu, mask, P, False, 0.0, 0.0, seed=5, step=7)
    ref = normalize_slices_reference((0.5 * (2 * mu - 1 + 1)).clamp(0, 1).view(E, -1, P).cpu().double(), 0.1, 2)
    torch.testing.assert_close(out.cpu(), ref.float().view(E, A), rtol=1e-6, atol=1e-6)


def test_explore_noise_independent_of_slice_shape():
    """The raw noisy weights (no threshold / normalisation passes) depend only on (seed, step, flat index) above 32
    destinations: the octet path (n_pad 200: two slices per wave, 8 weights per lane) and the one-slice-per-wave path
    (n_pad 40) give identical bits for the same action block.  (n_pad <= 32 keeps the round-5 stream.)"""
    torch.manual_seed(3)
    E, A = 4, 200 * 3 * 200
    mu = torch.rand(E, A, device=DEV)
    mask = torch.ones(E, A, device=DEV)
    for warm in (True, False):
        a = explore_postprocess(mu, mask, 200, warm, 0.0, 0.3, seed=9, step=4, threshold=0.0, passes=0)
        b = explore_postprocess(mu, mask, 40, warm, 0.0, 0.3, seed=9, step=4, threshold=0.0, passes=0)
        assert torch.equal(a, b)


@pytest.mark.parametrize("P", [40, 200])
def test_explore_octet_stream_is_philox4x32_10(P):
    """The wave kernels' noise words are Philox4x32-10 (key = (seed, step), counter = flat index / 8; the device
    rounds use host round keys and one v_bitop3 xor3 per key mix) -- pinned against the pure-Python Philox of
    tests/test_replay.py through the warm-up uniforms: weight f = 16-bit half (f & 1) of word (f & 7) / 2, * 2^-16."""
    from tests.test_replay import philox4x32_10
    E, A = 2, P * 3 * P
    mask = torch.ones(E, A, device=DEV)
    mu = torch.zeros(E, A, device=DEV)
    u = explore_postprocess(mu, mask, P, True, 0.0, 0.3, seed=77, step=12, threshold=0.0, passes=0).cpu().flatten()
    for f in list(range(0, 64)) + list(range(E * A - 40, E * A)) + [12345 % (E * A), 99999 % (E * A)]:
        w = philox4x32_10(77, 12, f >> 3)[(f & 7) >> 1]
        h = (w >> 16) if f & 1 else (w & 0xffff)
        assert float(u[f]) == h / 65536.0, f


@pytest.mark.parametrize("P,n", [(50, 50), (200, 200), (200, 131), (64, 7)])
def test_explore_noisy_rows_match_reference_postprocess(P, n):
    """Noisy rows against the reference post-processing (fp64, simple_ddpg.py:338-395) of the same raw noisy
    weights (the passes=0 output).  mu mixes flat rows (pass 2 zeroes them: the kernel's early uniform exit)
    with one-hot rows (a weight stays >= 0.1 through pass 2: the general loop), so both paths are compared
    (noise sigma 0.1: at 0.3 the noise alone spreads a one-hot row at 200 destinations below the threshold)."""
    torch.manual_seed(4)
    E, A = 8, P * 3 * P
    mask = torch.zeros(E, P, 3, P, device=DEV)
    mask[:, :n, :, :n] = 1
    mask = mask.view(E, A)
    mu = (torch.rand(E, A // P, P, device=DEV) * 0.6).view(E, A)
    hot = torch.zeros(E, A // P, P, device=DEV)
    hot[:, ::2, 0] = 1.0  # every other row: one destination near 1, the rest at 0
    mu = torch.where(hot.view(E, A).bool() | (torch.arange(A // P, device=DEV) % 2 == 1).repeat_interleave(P)[None],
                     torch.where(hot.view(E, A).bool(), torch.ones_like(mu), torch.zeros_like(mu)), mu) * mask
    for warm in (True, False):
        raw = explore_postprocess(mu, mask, P, warm, 0.0, 0.1, seed=11, step=3, threshold=0.0, passes=0)
        out = explore_postprocess(mu, mask, P, warm, 0.0, 0.1, seed=11, step=3)
        ref = normalize_slices_reference(raw.view(E, -1, P).cpu().double(), 0.1, 2).float()
        torch.testing.assert_close(out.cpu().view(E, -1, P), ref, rtol=1e-6, atol=1e-6)
        uniform = (ref.amax(-1) - ref.amin(-1)).abs() < 1e-6
        if not warm and n > 100:
            assert uniform.any() and (~uniform).any(), "both kernel paths exercised"


@pytest.mark.parametrize("P", [20, 40, 200])
def test_explore_noise_is_standard_normal(P):
    """The raw exploration noise (passes 0, mu = 0.5, sigma 0.1: weight = 0.5 + 0.05 z) is standard normal in every
    kernel family (lanes / one slice per wave / two slices per wave): moments and tail mass of ~1.2M samples, and
    the warm-up uniforms are U[0, 1)."""
    E, A = 4, P * 3 * P if P > 20 else 20 * 3 * 200
    while E * A < 1_000_000:
        E *= 2
    mu = torch.full((E, A), 0.5, device=DEV)
    mask = torch.ones(E, A, device=DEV)
    a = explore_postprocess(mu, mask, P, False, 0.0, 0.1, seed=21, step=5, threshold=0.0, passes=0)
    z = ((a.double() - 0.5) / 0.05).flatten()
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01
    assert abs(float((z ** 4).mean()) - 3.0) < 0.1                       # Gaussian kurtosis
    assert abs(float((z.abs() > 2).double().mean()) - 0.0455) < 0.002    # two-sigma tail mass
    assert abs(float(torch.corrcoef(torch.stack([z[0::2], z[1::2]]))[0, 1])) < 0.01  # Box-Muller pair partners
    u = explore_postprocess(mu, mask, P, True, 0.0, 0.1, seed=21, step=5, threshold=0.0, passes=0).double().flatten()
    assert float(u.min()) >= 0.0 and float(u.max()) < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.005 and abs(float(u.var()) - 1.0 / 12.0) < 0.002


@pytest.mark.parametrize("P,n,R", [(200, 200, 600), (200, 131, 7), (256, 256, 9)])
def test_explore_octet_kernel_matches_slice_kernel(P, n, R, monkeypatch):
    """The two-slices-per-wave exploration kernel (n_pad > 128, n_pad % 8 == 0: one Philox draw per 8 weights per
    lane) equals the one-slice-per-wave kernel bit for bit -- raw weights (passes 0), post-processed rows with both
    the early uniform exit and the general loop, warm-up and noisy; an odd row count leaves a half-wave idle."""
    torch.manual_seed(5)
    E, A = 6, P * R
    T = 2
    tab = torch.zeros(T, R, P, device=DEV)
    tab[:, :, :n] = 1
    tab[1, :, n // 2:] = 0
    topo = torch.tensor([0, 1, 1, 0, 1, 0], device=DEV)
    mu = torch.rand(E, R, P, device=DEV) * 0.6
    mu[:, ::3] = 0
    mu[:, ::3, 0] = 1.0  # one-hot rows: the general loop
    mu = mu.view(E, A)
    tab = tab.view(T, A)
    for warm in (True, False):
        for kw in (dict(threshold=0.0, passes=0), dict()):
            monkeypatch.setenv("GSC_EXPLORE_OCT", "1")
            a = explore_postprocess(mu, tab, P, warm, 0.0, 0.1, seed=3, step=9, topo=topo, **kw)
            monkeypatch.setenv("GSC_EXPLORE_OCT", "0")
            b = explore_postprocess(mu, tab, P, warm, 0.0, 0.1, seed=3, step=9, topo=topo, **kw)
            assert torch.equal(a, b), (warm, kw)


@pytest.mark.parametrize("N,H,T,A", [(256, 22, 3, 360000), (64, 22, 1, 1728), (33, 5, 4, 1001)])
def test_first_layer_grad_rows_kernel_bitwise(N, H, T, A, monkeypatch):
    """First-layer gradient dW[n] = [tmp[n][:H] | sum_t tmp[n][H+1+t] mask_t], db[n] = tmp[n][H] (csrc/ops/mlp.hip):
    the row-grid kernel equals the grid-stride kernel bit for bit and fp32 PyTorch to rounding."""
    from gsc_amd.native import load
    nat = load()
    g = torch.Generator(device="cuda").manual_seed(2)
    tmp = torch.randn(N, H + 1 + T, device="cuda", generator=g)
    mask = (torch.rand(T, A + 3, device="cuda", generator=g) > 0.4).float()
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("GSC_FLG_ROWS", v)
        gW = torch.full((N, H + A + 5), float("nan"), device="cuda")
        gb = torch.full((N,), float("nan"), device="cuda")
        nat.first_layer_grad(tmp.data_ptr(), N, H, T, A, mask.data_ptr(), mask.stride(0), gW.data_ptr(), gW.stride(0),
                             gb.data_ptr(), torch.cuda.current_stream().cuda_stream)
        outs.append((gW, gb))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0][:, :H + A], outs[1][0][:, :H + A]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.isnan(outs[1][0][:, H + A:]).all()
    ref = torch.cat([tmp[:, :H], tmp[:, H + 1:] @ mask[:, :A]], 1)
    torch.testing.assert_close(outs[1][0][:, :H + A], ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(outs[1][1], tmp[:, H])


@pytest.mark.parametrize("R,C,masked", [(64, 360000, True), (3, 1001, False), (70, 257, True)])
def test_copy2d_rows_kernel_bitwise(R, C, masked, monkeypatch):
    """copy2d (dst = bf16(src * colmask), strided rows): the row-grid kernel equals the grid-stride kernel bit for bit
    and the PyTorch product."""
    from gsc_amd.native import load
    nat = load()
    g = torch.Generator(device="cuda").manual_seed(3)
    src = torch.randn(R, C + 9, device="cuda", generator=g).bfloat16()
    cm = (torch.rand(C, device="cuda", generator=g) > 0.5).float()
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("GSC_COPY2D_ROWS", v)
        dst = torch.full((R, C + 5), float("nan"), device="cuda").bfloat16()
        nat.copy2d(src.data_ptr() + 2 * 3, src.stride(0), dst.data_ptr(), dst.stride(0), R, C,
                   cm.data_ptr() if masked else 0, torch.cuda.current_stream().cuda_stream)
        outs.append(dst)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][:, :C].view(torch.int16), outs[1][:, :C].view(torch.int16))
    ref = (src[:, 3:3 + C].float() * (cm if masked else 1.0)).bfloat16()
    assert torch.equal(outs[1][:, :C].view(torch.int16), ref.view(torch.int16))


def test_splitk_linear_matches_linear():
    """Split-K weight gradient == plain GEMM gradient (fp32 reference, bf16 autocast tolerance)."""
    from gsc_amd.ops.linear import linear
    torch.manual_seed(0)
    x = torch.randn(25600, 1728, device=DEV, requires_grad=True)
    w = torch.randn(64, 1728, device=DEV, requires_grad=True)
    b = torch.randn(64, device=DEV, requires_grad=True)
    g = torch.randn(25600, 64, device=DEV)
    ref = torch.autograd.grad((torch.nn.functional.linear(x, w, b) * g).sum(), (x, w, b))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = linear(x, w, b)
    assert out.dtype == torch.bfloat16
    got = torch.autograd.grad((out.float() * g).sum(), (x, w, b))
    for r, o in zip(ref, got):
        assert o.dtype == r.dtype
        assert (o - r).abs().max() <= 2e-2 * r.abs().max()


@pytest.mark.parametrize("M,K,A,J,T", [(300, 256, 1000, 64, 3), (128, 128, 4096, 48, 1), (77, 64, 136, 64, 4),
                                       (300, 256, 1001, 64, 2), (16384, 256, 8200, 64, 3)])
def test_actor_proj_matches_reference(M, K, A, J, T):
    """Fused actor output layer + critic action projection (csrc/ops/actor_proj.hip) against fp32
    PyTorch: Z = bf16(clamp((H W^T + b) * mask[topo], -1, 1)) Wa^T (edge tiles in M, A and J).
    A % 8 != 0: Wa rows zero-padded to a multiple of 8 columns (the caller's contract); 16,384 rows x
    129 tiles: the large-batch, long-action-space split (8 splits)."""
    from gsc_amd.native import load
    nat = load()
    g = torch.Generator(device="cuda").manual_seed(0)
    h = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    w = (torch.randn(A, K, device="cuda", generator=g) * 0.1).bfloat16()
    b = torch.randn(A, device="cuda", generator=g) * 0.1
    mask = (torch.rand(T, A, device="cuda", generator=g) > 0.3).float()
    topo = torch.randint(0, T, (M,), device="cuda", generator=g, dtype=torch.int32)
    wa = (torch.randn(J, A, device="cuda", generator=g) * 0.05).bfloat16()
    wa_pad = torch.zeros(J, -(-A // 8) * 8, device="cuda", dtype=torch.bfloat16)
    wa_pad[:, :A] = wa
    slabs = torch.empty(1 << 24, device="cuda")
    z = torch.full((M, 80), float("nan"), device="cuda")
    nat.actor_proj(h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), b.data_ptr(), mask.data_ptr(), mask.stride(0),
                   T, topo.data_ptr(), wa_pad.data_ptr(), wa_pad.stride(0), M, K, A, J, -1.0, 1.0, slabs.data_ptr(),
                   slabs.numel(), z.data_ptr(), z.stride(0), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    p = ((h.float() @ w.float().t() + b) * mask[topo.long()]).clamp(-1, 1).bfloat16().float()
    ref = p @ wa.float().t()
    err = float((z[:, :J] - ref).norm() / ref.norm())
    assert err < 5e-3, err
    assert torch.isnan(z[:, J:]).all()          # only the J columns are written


@pytest.mark.parametrize("T,N,A", [(3, 256, 360000), (1, 64, 1875), (2, 64, 1001)])
def test_rowdot_mask_fold_bits_match_fp32(T, N, A, monkeypatch):
    """Mask fold out[t][n] = sum_a mask[t][a] W[n][a] (csrc/ops/mlp.hip rowdot): the packed-bit mask variant on
    the 4-byte pair loop equals the fp32-mask variant (0/1 weights: identical terms); the 16-byte-load bit variant
    (rowdot_bits8_kernel, W rows starting 3 elements past a 16-byte boundary: head, vectors, tail) matches them to
    fp32 summation order; all match fp32 PyTorch."""
    from gsc_amd.agents.native_update import mask_bits
    from gsc_amd.native import load
    nat = load()
    g = torch.Generator(device="cuda").manual_seed(1)
    masks = (torch.rand(T, A, device="cuda", generator=g) > 0.5).float()
    W = (torch.randn(N, A + (8 if T == 3 else 7), device="cuda", generator=g) * 0.05).bfloat16()  # pair / scalar path
    bits = mask_bits(masks)
    ws = torch.zeros(64 * T * N, device="cuda")
    outs = []
    monkeypatch.setenv("GSC_ROWDOT_VEC", "0")
    for xb in (None, bits, bits):
        if len(outs) == 2:
            monkeypatch.setenv("GSC_ROWDOT_VEC", "1")
        o = torch.full((T, N), float("nan"), device="cuda")
        nat.rowdot(masks.data_ptr(), masks.stride(0), T, W.data_ptr(), W.stride(0), N, A, o.data_ptr(), o.stride(0),
                   torch.cuda.current_stream().cuda_stream, ws.data_ptr(), ws.numel(),
                   xb.data_ptr() if xb is not None else 0, xb.shape[1] if xb is not None else 0)
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    torch.testing.assert_close(outs[2], outs[1], rtol=1e-5, atol=1e-5)
    ref = masks @ W[:, :A].float().t()
    assert float((outs[1] - ref).norm() / ref.norm()) < 1e-5
    assert float((outs[2] - ref).norm() / ref.norm()) < 1e-5
    # misaligned row slices (the first layer's mask block starts at column H): 16-byte path vs fp32 PyTorch
    Wm = W[:, 3:]
    o = torch.full((T, N), float("nan"), device="cuda")
    nat.rowdot(masks.data_ptr(), masks.stride(0), T, Wm.data_ptr(), Wm.stride(0), N, A - 3, o.data_ptr(), o.stride(0),
               torch.cuda.current_stream().cuda_stream, ws.data_ptr(), ws.numel(), 0, 0)
    bm = mask_bits(masks[:, :A - 3].contiguous())
    o8 = torch.full((T, N), float("nan"), device="cuda")
    nat.rowdot(masks.data_ptr(), masks.stride(0), T, Wm.data_ptr(), Wm.stride(0), N, A - 3, o8.data_ptr(),
               o8.stride(0), torch.cuda.current_stream().cuda_stream, ws.data_ptr(), ws.numel(), bm.data_ptr(),
               bm.shape[1])
    torch.cuda.synchronize()
    ref_m = masks[:, :A - 3] @ Wm[:, :A - 3].float().t()
    assert float((o8 - ref_m).norm() / ref_m.norm()) < 1e-5
    torch.testing.assert_close(o8, o, rtol=1e-5, atol=1e-5)
