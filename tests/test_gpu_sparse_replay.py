"""GPU: sparse replayed actions (csrc/ops/sparse_act.hip) -- the record ring decodes to exactly the dense bf16
rows, the critic's two action products on the records match fp32 dense products, and the batched trainer on a
200-node topology with the sparse ring tracks the dense ring's learner."""
import os

import numpy as np
import pytest
import torch
import yaml

from gsc_amd.agents.replay import DeviceReplay
from gsc_amd.ops.explore import explore_postprocess
from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu


def _post_processed(E, R, P, seed, peaked=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mu = torch.rand(E, R * P, device="cuda", generator=g)
    if peaked:
        mu *= 0.2
        top = torch.randint(0, P, (E, R, 2), device="cuda", generator=g)
        mu.view(E, R, P).scatter_(-1, top, 0.95)
    mask = torch.ones(1, R * P, device="cuda")
    topo = torch.zeros(E, dtype=torch.int64, device="cuda")
    return explore_postprocess(mu, mask, P, False, 0.0, 0.3, seed, 1, topo=topo)


@pytest.mark.parametrize("P", [52, 200])
def test_sparse_compress_kernels_write_identical_records(P, monkeypatch):
    """The 16-byte-load compress kernel (P % 4 == 0) writes the same record words -- base, count, exceptions in
    ascending destination order -- as the lane-strided one, uniform and peaked rows alike."""
    E, R, cap = 16, 24, 40
    rings = []
    for v in ("0", "1"):
        monkeypatch.setenv("GSC_SP_COMPRESS4", v)
        rep = DeviceReplay(cap, P, 3, R * P, "cuda", action_dtype=torch.bfloat16, sparse_rows=R)
        for k in range(2):
            a = _post_processed(E, R, P, 20 + k, peaked=k == 1)
            z = torch.zeros(E, P, 3, device="cuda")
            rep.add(z, torch.zeros(E, dtype=torch.int64, device="cuda"), a, torch.zeros(E, device="cuda"), z,
                    torch.zeros(E, device="cuda"))
        torch.cuda.synchronize()
        rep.check_sparse()
        rings.append(rep.actions[:2 * E].clone())
    assert torch.equal(rings[0], rings[1])


@pytest.mark.parametrize("P", [50, 200])
def test_sparse_ring_decodes_to_dense_bf16(P):
    E, R, cap = 16, 24, 40
    rep = DeviceReplay(cap, P, 3, R * P, "cuda", action_dtype=torch.bfloat16, sparse_rows=R)
    want = []
    for k in range(3):   # wraps the ring: 48 rows into 40 slots
        a = _post_processed(E, R, P, 10 + k, peaked=k == 1)
        want.append(a)
        z = torch.zeros(E, P, 3, device="cuda")
        rep.add(z, torch.zeros(E, dtype=torch.int64, device="cuda"), a, torch.zeros(E, device="cuda"), z,
                torch.zeros(E, device="cuda"))
    torch.cuda.synchronize()
    rep.check_sparse()
    rows = torch.arange(0, 40, device="cuda")
    got = rep.dense_actions(rows)
    # slots 0-15 add 1, 16-31 add 2, 32-39 + 0-7 add 3 (wrapped)
    ref = torch.cat([want[2][8:], want[0][8:], want[1], want[2][:8]]).to(torch.bfloat16)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    head = (rep.actions[:, :, 0].long() >> 16) & 0xffff
    assert int(head.max()) <= 11


@pytest.mark.parametrize("P", [50, 200])
def test_sparse_critic_products_match_fp32_dense(P):
    """Both MFMA products on the records (P = 200: 16-byte W_a loads; P = 50: element loads and record blocks that
    straddle 8-column chunks) against fp32 dense products of the decoded rows."""
    from gsc_amd.native import load
    nat = load()
    E, R, c1, B = 64, 36, 64, 600   # B not a multiple of 256 / 64: partial sample tiles
    A = R * P
    rep = DeviceReplay(E, P, 3, A, "cuda", action_dtype=torch.bfloat16, sparse_rows=R)
    a = torch.cat([_post_processed(E // 2, R, P, 3), _post_processed(E // 2, R, P, 4, peaked=True)])
    z = torch.zeros(E, P, 3, device="cuda")
    rep.add(z, torch.zeros(E, dtype=torch.int64, device="cuda"), a, torch.zeros(E, device="cuda"), z,
            torch.zeros(E, device="cuda"))
    g = torch.Generator(device="cuda").manual_seed(5)
    rows = torch.randint(0, E, (B,), device="cuda", dtype=torch.int32, generator=g)
    lda = A + 8
    wa = (torch.randn(c1, lda, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    dh0 = (torch.randn(B, c1, device="cuda", generator=g)).to(torch.bfloat16)
    S = 4
    part = torch.zeros(S, B, c1, device="cuda")
    wsum = torch.empty(R * c1, dtype=torch.int32, device="cuda")
    hacc = torch.zeros(B, c1, device="cuda")
    gw = torch.zeros(c1, A, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nat.sparse_fwd(rep.actions.data_ptr(), rows.data_ptr(), B, R, P, wa.data_ptr(), lda, c1, wsum.data_ptr(), part.data_ptr(), S, s)
    nat.splitk_reduce(part.data_ptr(), B * c1, S, B, c1, c1, hacc.data_ptr(), c1, 1.0, 0, s)
    nat.sparse_wgrad(rep.actions.data_ptr(), rows.data_ptr(), B, R, P, dh0.data_ptr(), c1, c1, gw.data_ptr(), A, s)
    torch.cuda.synchronize()
    dense = rep.dense_actions(rows.long()).float()                 # [B, A]
    h_ref = dense @ wa[:, :A].float().t()
    gw_ref = dh0.float().t() @ dense
    eh = ((hacc - h_ref).norm() / h_ref.norm()).item()
    eg = ((gw - gw_ref).norm() / gw_ref.norm()).item()
    print(f"rel err forward {eh:.2e} weight grad {eg:.2e}")
    assert eh < 1e-3 and eg < 1e-3, (eh, eg)


def test_trainer_sparse_ring_tracks_dense_ring():
    """syn200 topologies (A = 360,000) on the batched trainer: a few updates with the sparse ring and with the
    dense bf16 ring from identical seeds -- the same transitions are replayed, so the critic parameters agree
    to the factored products' rounding."""
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    nets = [cfg_path("networks", "synthetic", f"syn200-in16-cap1-3-s{i}.graphml") for i in range(2)]
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "agent_syn200.yaml")))
    cfg["episode_steps"] = 5
    out = {}
    for mode in ("1", "0"):
        os.environ["GSC_SPARSE_REPLAY"] = mode
        try:
            sim = load_batched_from_paths(nets, cfg_path("service_functions", "abc-3sfc.yaml"),
                                          cfg_path("config", "simulator", "sample_config.yaml"), cfg, 16,
                                          device="cuda", seed=7)
            tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=16, batch_size=256, learning_starts=2, seed=3,
                                                        check_every=0, replay_capacity=64, overlap_sim=False),
                                network_schedule=[0, 1], period=1)
            assert bool(tr.replay.sparse_rows) == (mode == "1")
            for _ in range(5):
                tr.step()
            torch.cuda.synchronize()
            tr.replay.check_sparse()
            out[mode] = (tr.learner.critic_flat.view().clone(), tr.learner.actor_flat.view().clone(),
                         tr.learner.updates)
        finally:
            os.environ.pop("GSC_SPARSE_REPLAY", None)
    assert out["1"][2] == out["0"][2] >= 3
    for k in (0, 1):
        d = (out["1"][k] - out["0"][k]).abs().max().item()
        assert d < 5e-3, (k, d)   # a few Adam steps of lr 1e-3 from identical replays
