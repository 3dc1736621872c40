"""GPU: the native DDPG update (MFMA GEMMs + fused epilogues + MFMA GNN + head/loss kernels + fused
Adam) against the CPU fp32 autograd learner, from identical initial weights and batches.

Checks, per parameter tensor, the gradients of the first update (relative L2 error, bf16 operands)
and, over three updates, the losses and the parameter trajectories (cosine of the deltas)."""
import numpy as np
import pytest
import torch
import yaml

from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu

ABILENE = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
# three topologies with different node counts (11, 15, 14): different action masks per topology
THREE = [ABILENE, cfg_path("networks", "Claranet_n15_e18", "Claranet-in4-cap1.graphml"),
         cfg_path("networks", "Compuserve_n14_e17", "Compuserve-in4-cap1.graphml")]


def _cfg(actor=(256,), critic=(64,)):
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    cfg["actor_hidden_layer_nodes"] = list(actor)
    cfg["critic_hidden_layer_nodes"] = list(critic)
    return cfg


def _batch(B, T, device, seed=11, P=24):
    from gsc_amd.agents import Batch
    g = torch.Generator().manual_seed(seed)
    obs = torch.rand(B, P, 3, generator=g)
    obs[:, 11:] = 0
    nxt = torch.rand(B, P, 3, generator=g)
    nxt[:, 11:] = 0
    act = torch.rand(B, P * 3 * P, generator=g)
    topo = torch.randint(0, T, (B,), generator=g)
    b = Batch(obs, topo, act, torch.rand(B, generator=g) - 0.5, nxt, (torch.rand(B, generator=g) < 0.2).float())
    if device == "cpu":
        return b
    return Batch(*(t.to(device) for t in b[:2]), b.actions.to(device).bfloat16(), *(t.to(device) for t in b[3:]))


def _learners(cfg, T, P=24, nets=None, C=1):
    from gsc_amd.agents import DDPGLearner
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GraphSet
    if nets is not None:
        topos = [load_topology(p) for p in nets]
    else:
        topos = [load_topology(ABILENE)] * T if T < 3 else [load_topology(p) for p in THREE]
    A = P * C * 3 * P
    ref = DDPGLearner(cfg, 3, A, GraphSet(topos, P, "cpu"), C, 3, "cpu", amp_bf16=False, seed=3)
    gpu = DDPGLearner(cfg, 3, A, GraphSet(topos, P, "cuda"), C, 3, "cuda", seed=3)
    assert gpu.native_ok
    assert torch.equal(ref.actor_flat.flat, gpu.actor_flat.flat.cpu())
    return ref, gpu


def _per_param_err(flat_ref, flat_gpu, what="grad"):
    out = {}
    for name, p, o in zip(flat_ref.names, flat_ref.params, flat_ref.offsets):
        n = p.numel()
        a = getattr(flat_ref, what)[o:o + n]
        b = getattr(flat_gpu, what)[o:o + n].cpu()
        den = a.norm().item()
        out[name] = (a - b).norm().item() / max(den, 1e-12) if den > 1e-8 else (a - b).norm().item()
    return out


@pytest.mark.parametrize("case", ["composed", "two_topologies", "three_topologies", "deep", "odd_actions", "sigmoid",
                                  "sigmoid_two_topologies"])
def test_native_update_matches_fp32_reference(case):
    """Tolerance: per tensor max(3 %, 2.5x the error of the PyTorch bf16-autocast path on the same
    batch) -- deeper nets amplify bf16 rounding through ReLU gates, for either implementation.  The
    deep case's floor is 4 %: the embedder gradients inherit the ~3.5 % bf16 error of the embedding
    gradient after three hidden layers (every embedder tensor, against 2 % for autocast), and the
    fp32-accumulated bias sums of one tensor land at 3.2 % where autocast happens to reach 0.8 %.
    odd_actions: n_pad 25, A = 1,875 (A % 8 != 0): the fused TD-target projection reads zero-padded
    critic action rows.  three_topologies (different action masks): the critic is frozen (learning rate 0).  With it
    training, the first critic step makes the trajectories chaotic -- Adam's first step is lr * sign(g)
    for every weight and the 1,728 action-block weights of each critic unit move coherently (qf1 jumps
    0.09 -> 4.2) -- so the actor gradients of any two bf16 implementations then differ by 10-20 %
    (autocast included); through a frozen critic ours and autocast agree per tensor (within 0.5 %
    absolute of each other against fp32, scripts/diag/learner_t3.py)."""
    T = {"two_topologies": 2, "three_topologies": 3}.get(case, 1)
    P = 25 if case == "odd_actions" else 24         # A = 1,875: A % 8 != 0 (padded action rows)
    cfg = _cfg(actor=(128, 96), critic=(64, 32)) if case == "deep" else _cfg()
    if case.startswith("sigmoid"):
        # bounded actor: materialised [B, A] output with the sigmoid epilogue and its in-place backward gate
        cfg["actor_output_activation"] = "sigmoid"
        T = 2 if case == "sigmoid_two_topologies" else 1
    ref, gpu = _learners(cfg, T, P)
    if case.startswith("sigmoid"):
        nu = gpu.native_update(512)
        assert nu.squash and not nu.compose and not nu.fuse_target
    _, auto = _learners(cfg, T, P)
    auto.native_ok = False                               # autograd + hipBLASLt bf16 path
    if case == "three_topologies":
        for l in (ref, gpu, auto):
            l.critic_opt.lr = 0.0
    B = 512
    for k in range(3):
        bc, bg = _batch(B, T, "cpu", seed=11 + k, P=P), _batch(B, T, "cuda", seed=11 + k, P=P)
        ref.update(bc)
        gpu.update(bg)
        auto.update(bg)
        torch.cuda.synchronize()
        if k == 0:
            for nm in ("critic_flat", "actor_flat"):
                fr, fg, fa = getattr(ref, nm), getattr(gpu, nm), getattr(auto, nm)
                e_nat, e_auto = _per_param_err(fr, fg), _per_param_err(fr, fa)
                print(case, nm, {n: (round(e_nat[n], 4), round(e_auto[n], 4)) for n in e_nat})
                floor = 0.04 if case == "deep" else 0.03
                bad = {n: (e, e_auto[n]) for n, e in e_nat.items() if e > max(floor, 2.5 * e_auto[n])}
                assert not bad, bad
                tot = ((fr.grad - fg.grad.cpu()).norm() / fr.grad.norm()).item()
                tot_a = ((fr.grad - fa.grad.cpu()).norm() / fr.grad.norm()).item()
                assert tot < max(0.03, 2.5 * tot_a), (tot, tot_a)
        for key in ("qf1_loss", "actor_loss", "qf1_values"):
            r, g, au = float(ref.last[key]), float(gpu.last[key]), float(auto.last[key])
            assert abs(r - g) <= max(0.03 * abs(r) + 1e-3, 2.5 * abs(r - au)), (k, key, r, g, au)
    # parameter trajectories: delta directions agree
    a0, _ = _learners(cfg, T, P)
    for nm in ("actor_flat", "critic_flat"):
        fr, fg, fa, f0 = (getattr(x, nm) for x in (ref, gpu, auto, a0))
        dr = fr.flat - f0.flat
        cos = torch.nn.functional.cosine_similarity(dr, fg.flat.cpu() - f0.flat, dim=0).item()
        if float(dr.norm()) == 0.0:                       # frozen critic
            continue
        cos_a = torch.nn.functional.cosine_similarity(dr, fa.flat.cpu() - f0.flat, dim=0).item()
        print(case, nm, "trajectory cosine", round(cos, 4), "autocast", round(cos_a, 4))
        assert cos > (0.97 if case != "deep" else 0.9), (cos, cos_a)


def test_composed_matches_materialised(monkeypatch):
    """Three topologies with different action masks: the composed actor loss (rows expanded into T
    blocks, Mc_t = W_a diag(m_t) W) and the materialised [B, A] actor output are the same function --
    identical critic gradients, actor gradients within bf16 re-association (< 2 % per tensor), the
    same losses over three updates."""
    cfg = _cfg()
    _, comp = _learners(cfg, 3)
    monkeypatch.setenv("GSC_COMPOSE", "0")
    _, mat = _learners(cfg, 3)
    assert not mat.native_update(512).compose      # built lazily: decided while the variable is set
    monkeypatch.delenv("GSC_COMPOSE")
    assert comp.native_update(512).compose
    for k in range(3):
        bg = _batch(512, 3, "cuda", seed=11 + k)
        comp.update(bg)
        mat.update(bg)
        torch.cuda.synchronize()
        if k == 0:
            for nm, tol in (("critic_flat", 1e-6), ("actor_flat", 0.02)):
                fm, fc = getattr(mat, nm), getattr(comp, nm)
                for n, p, o in zip(fm.names, fm.params, fm.offsets):
                    gm, gc = fm.grad[o:o + p.numel()], fc.grad[o:o + p.numel()]
                    err = float((gm - gc).norm() / gm.norm().clamp_min(1e-12))
                    assert err < tol, (nm, n, err)
        for key in ("qf1_loss", "actor_loss", "qf1_values"):
            a, b = float(comp.last[key]), float(mat.last[key])
            assert abs(a - b) <= 0.01 * abs(a) + 1e-4, (k, key, a, b)


def test_native_update_graphed_matches_eager():
    """The captured HIP-graph replay computes exactly what the eager native stages compute."""
    cfg = _cfg()
    _, g1 = _learners(cfg, 1)
    _, g2 = _learners(cfg, 1)
    b = _batch(1024, 1, "cuda")
    for _ in range(4):
        g1.update(b)
        g2.update_graphed(b, warmup=1)
    torch.cuda.synchronize()
    assert torch.equal(g1.actor_flat.flat, g2.actor_flat.flat)
    assert torch.equal(g1.critic_flat.flat, g2.critic_flat.flat)
    assert torch.equal(g1.target_actor_flat.flat, g2.target_actor_flat.flat)


@pytest.mark.parametrize("T,act", [(1, "none"), (2, "none"), (2, "sigmoid")])
def test_native_act_matches_fp32_module(T, act):
    """Acting forward on the native kernels (embedder, folded mask block, hidden, masked output; the
    sigmoid epilogue for a bounded actor) against the fp32 PyTorch actor on the same weights."""
    cfg = _cfg()
    cfg["actor_output_activation"] = act
    ref, gpu = _learners(cfg, T)
    E = 300
    gpu.enable_native_act(E)
    assert gpu._act_native is not None
    b = _batch(E, T, "cpu", seed=5)
    with torch.no_grad():
        want = ref.actor(b.obs, b.topo, ref.graphs, ref.masks)
    got = gpu.act(b.obs.cuda().contiguous(), b.topo.cuda()).cpu()
    err = ((got - want).norm() / want.norm()).item()
    assert err < 0.02, err
    # masked entries (padding nodes / other topologies' rows) are exactly zero
    m = ref.masks[b.topo]
    assert torch.equal(got * (1 - m), torch.zeros_like(got))


def test_native_act_follows_graphed_updates():
    """The acting forward's folded mask block is refreshed by the (captured) update after each actor
    step: after several graphed updates the native act still matches the fp32 actor module on the
    updated weights (the module's parameters alias the learner's flat buffer)."""
    cfg = _cfg()
    _, gpu = _learners(cfg, 2)
    E = 300
    gpu.enable_native_act(E)
    obs = _batch(E, 2, "cuda", seed=5)
    gpu.act(obs.obs.contiguous(), obs.topo)            # first act computes the fold itself
    b = _batch(1024, 2, "cuda", seed=7)
    for _ in range(4):                                 # 1 eager warm-up, capture, replays
        gpu.update_graphed(b, warmup=1)
    torch.cuda.synchronize()
    assert gpu._act_native.rowtab_owned
    got = gpu.act(obs.obs.contiguous(), obs.topo)
    with torch.no_grad():
        want = gpu.actor(obs.obs, obs.topo, gpu.graphs, gpu.masks).float()
    err = ((got - want).norm() / want.norm()).item()
    assert err < 0.02, err


def test_native_update_reads_replay_rows_in_place():
    """The critic's action GEMMs reading the sampled replay-ring rows in place (row-indexed operands,
    DeviceReplay.sample(actions=False)) compute exactly the update of the gathered [B, A] batch."""
    from gsc_amd.agents.replay import DeviceReplay
    cfg = _cfg()
    _, g1 = _learners(cfg, 2)
    _, g2 = _learners(cfg, 2)
    A = 24 * 3 * 24
    rb = DeviceReplay(2000, 24, 3, A, "cuda", action_dtype=torch.bfloat16, seed=3, action_row_align=8)
    src = _batch(1000, 2, "cpu", seed=9)
    for k in range(2):
        sl = slice(500 * k, 500 * (k + 1))
        rb.add(src.obs[sl].cuda(), src.topo[sl].cuda(), src.actions[sl].cuda(), src.rewards[sl].cuda(),
               src.next_obs[sl].cuda(), src.dones[sl].cuda())
    B = 512
    for _ in range(2):
        b1 = rb.sample(B)                                        # gathered actions
        rb.state[2] -= 1                                         # same Philox draw again
        b2 = rb.sample(B, actions=False)                         # actions = the ring
        assert b2.actions is rb.actions
        g1.update(b1)
        g2.native_update(B).act_rows = rb.indices(B)
        g2.update(b2)
    torch.cuda.synchronize()
    for nm in ("critic_flat", "actor_flat", "target_critic_flat"):
        assert torch.equal(getattr(g1, nm).flat, getattr(g2, nm).flat), nm


SYN200 = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(3)]


@pytest.mark.parametrize("lg", ["1", "0"], ids=["fused-lg", "layer-wise"])
def test_native_update_matches_fp32_reference_200_nodes(lg, monkeypatch):
    """Config-5 shapes: n_pad 200, 3 SFCs x 3 SFs (A = 360,000), three 200-node topologies (different
    action masks), batch 256: the large-graph fused GNN kernels (GSC_GNN_LG=0: the layer-wise ones), the
    composed multi-topology actor loss
    (T c1 = 192 <= B), split-K action projections and the fused TD-target projection, against the fp32
    CPU autograd learner (first-update gradients per tensor, losses)."""
    monkeypatch.setenv("GSC_GNN_LG", lg)
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "agent_syn200.yaml")))
    P, C, T, B = 200, 3, 3, 256
    ref, gpu = _learners(cfg, T, P, nets=SYN200, C=C)
    _, auto = _learners(cfg, T, P, nets=SYN200, C=C)
    auto.native_ok = False
    for l in (ref, gpu, auto):
        l.critic_opt.lr = 0.0  # frozen critic (see the three_topologies case)
    nu = gpu.native_update(B)
    assert nu.compose and nu.fuse_target and nu.layerwise == (lg == "0")
    from gsc_amd.agents import Batch
    g = torch.Generator().manual_seed(5)
    topo = torch.arange(B) % T
    n = torch.tensor([gs_n for gs_n in ref.graphs.n_nodes.tolist()])[topo]
    obs = torch.rand(B, P, 3, generator=g) * (torch.arange(P)[None, :, None] < n[:, None, None])
    nxt = torch.rand(B, P, 3, generator=g) * (torch.arange(P)[None, :, None] < n[:, None, None])
    act = torch.rand(B, P * C * 3 * P, generator=g) * ref.masks[topo]
    bc = Batch(obs, topo, act, torch.rand(B, generator=g) - 0.5, nxt, (torch.rand(B, generator=g) < 0.2).float())
    bg = Batch(*(t.cuda() for t in bc[:2]), bc.actions.cuda().bfloat16(), *(t.cuda() for t in bc[3:]))
    ref.update(bc)
    gpu.update(bg)
    auto.update(bg)
    torch.cuda.synchronize()
    for nm in ("critic_flat", "actor_flat"):
        fr, fg, fa = getattr(ref, nm), getattr(gpu, nm), getattr(auto, nm)
        e_nat, e_auto = _per_param_err(fr, fg), _per_param_err(fr, fa)
        print("syn200", nm, {k: (round(e_nat[k], 4), round(e_auto[k], 4)) for k in e_nat})
        bad = {k: (e, e_auto[k]) for k, e in e_nat.items() if e > max(0.04, 2.5 * e_auto[k])}
        assert not bad, bad
    for key in ("qf1_loss", "actor_loss", "qf1_values"):
        r, gv, au = float(ref.last[key]), float(gpu.last[key]), float(auto.last[key])
        assert abs(r - gv) <= max(0.03 * abs(r) + 1e-3, 2.5 * abs(r - au)), (key, r, gv, au)
