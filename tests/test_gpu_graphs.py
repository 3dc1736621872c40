"""GPU: DDPG updates replayed from captured HIP graphs == eager updates (same batches, same init)."""
import pytest
import torch
import yaml

from gsc_amd.agents import Batch, DDPGLearner
from gsc_amd.coordsim.reader import load_topology
from gsc_amd.models import GraphSet
from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu


def _batches(n, B, dev):
    g = torch.Generator(device=dev).manual_seed(3)
    out = []
    for _ in range(n):
        obs = torch.rand(B, 24, 3, device=dev, generator=g)
        obs[:, 11:] = 0
        nxt = torch.rand(B, 24, 3, device=dev, generator=g)
        nxt[:, 11:] = 0
        out.append(Batch(obs, torch.zeros(B, dtype=torch.int64, device=dev),
                         torch.rand(B, 1728, device=dev, generator=g).to(torch.bfloat16),
                         torch.rand(B, device=dev, generator=g) - 0.5, nxt,
                         (torch.rand(B, device=dev, generator=g) < 0.1).float()))
    return out


def test_graphed_update_matches_eager():
    dev = "cuda"
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    gs = GraphSet([load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))], 24, dev)
    eager = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, seed=5)
    graphed = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, seed=5)
    assert torch.equal(eager.actor_flat.flat, graphed.actor_flat.flat)
    B = 512
    static = Batch(*(torch.empty_like(t) for t in _batches(1, B, dev)[0]))
    for b in _batches(6, B, dev):
        eager.update(b)
        for d, s in zip(static, b):
            d.copy_(s)
        graphed.update_graphed(static, warmup=2)
    torch.cuda.synchronize()
    assert graphed._graphs is not None and graphed.updates == eager.updates == 6
    for name in ("actor_flat", "critic_flat", "target_actor_flat", "target_critic_flat"):
        torch.testing.assert_close(getattr(graphed, name).flat, getattr(eager, name).flat, rtol=1e-5, atol=1e-6)
    assert graphed.actor_opt.step_count == eager.actor_opt.step_count == 6
    torch.testing.assert_close(graphed.last["qf1_loss"], eager.last["qf1_loss"], rtol=1e-5, atol=1e-6)


def test_bf16_shadows_match_autocast_casts():
    """Autograd path: updates using the bf16 parameter shadows == updates where autocast casts the fp32 weights."""
    dev = "cuda"
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    gs = GraphSet([load_topology(cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml"))], 24, dev)
    a = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, seed=9)
    b = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, seed=9)
    a.native_ok = b.native_ok = False  # autograd path: shadows vs autocast casts (the native path needs shadows)
    for fp in (b.actor_flat, b.critic_flat, b.target_actor_flat, b.target_critic_flat):
        fp.flat16 = None
        for p in fp.params:
            del p._bf16
    del b.masks._bf16
    for bt in _batches(3, 9000, dev):
        a.update(bt)
        b.update(bt)
    torch.cuda.synchronize()
    # identical except the actor's output bias, whose gradient the shadow path's composed projection
    # accumulates in fp32 where autocast's bf16 matmul rounds it (|diff| ~ 1e-6 after 3 Adam steps)
    for name in ("actor_flat", "critic_flat", "target_critic_flat"):
        torch.testing.assert_close(getattr(a, name).flat, getattr(b, name).flat, rtol=1e-5, atol=2e-5)
    n_b2 = a.actor.mlp.layers[-1].bias.numel()
    torch.testing.assert_close(a.actor_flat.flat[:a.actor_flat.numel - n_b2],
                               b.actor_flat.flat[:b.actor_flat.numel - n_b2], rtol=1e-5, atol=1e-6)
    # the shadow tracks the fp32 parameters exactly (round-to-nearest-even)
    assert torch.equal(a.actor_flat.flat16, a.actor_flat.flat.to(torch.bfloat16))
    assert torch.equal(a.target_critic_flat.flat16, a.target_critic_flat.flat.to(torch.bfloat16))
