"""The structure the sparse replay records rely on (csrc/ops/sparse_act.hip): every post-processed action row
(reference simple_ddpg.py:374-395, two passes of threshold 0.1 + renormalise) is, after the ring's bf16
rounding, either one value repeated (a uniform row, the first entry possibly off by the rounding residual) or
zero except for at most 11 entries.  Checked on the reference post-processing (CPU) over policies from diffuse
to concentrated; plus the record decoder."""
import numpy as np
import pytest
import torch

from gsc_amd.agents.replay import decompress_actions
from gsc_amd.ops.explore import explore_postprocess_reference

SLOTS = 11


def _exceptions(row_bf16: torch.Tensor):
    bits = row_bf16.view(torch.int16).to(torch.int32) & 0xffff
    m0 = int((bits != 0).sum())
    m1 = int((bits != bits[1]).sum())
    return min(m0, m1)


@pytest.mark.parametrize("P", [24, 50, 200])
@pytest.mark.parametrize("kind", ["diffuse", "peaked", "sparse", "warmup"])
def test_post_processed_rows_fit_sparse_records(P, kind):
    g = torch.Generator().manual_seed(P * 7 + len(kind))
    E, R = 4, 12
    if kind == "diffuse":
        mu = torch.rand(E, R * P, generator=g)
    elif kind == "peaked":      # a few large weights per row (a trained, concentrated policy)
        mu = torch.rand(E, R * P, generator=g) * 0.2
        top = torch.randint(0, P, (E, R, 3), generator=g)
        mu.view(E, R, P).scatter_(-1, top, 0.95)
    else:
        mu = (torch.rand(E, R * P, generator=g) > 0.9).float()
    mask = torch.ones(E, R * P)
    a = explore_postprocess_reference(mu, mask, P, kind == "warmup", 0.0, 0.3 if kind != "sparse" else 0.05, g)
    rows = a.to(torch.bfloat16).view(E * R, P)
    worst = max(_exceptions(r) for r in rows)
    assert worst <= SLOTS, (kind, P, worst)


def test_decompress_actions_reference():
    P, R = 20, 3
    rec = torch.zeros(2, R, 12, dtype=torch.int64)
    bf = lambda x: int(torch.tensor([x], dtype=torch.bfloat16).view(torch.int16).item()) & 0xffff
    u = bf(0.05)
    rec[0, 0, 0] = u | (1 << 16)                 # uniform row, first entry off
    rec[0, 0, 1] = 0 | (bf(0.0625) << 16)
    rec[0, 1, 0] = 0 | (2 << 16)                 # two exceptions on a zero base
    rec[0, 1, 1] = 3 | (bf(0.25) << 16)
    rec[0, 1, 2] = 17 | (bf(0.75) << 16)
    rec[0, 1, 3] = 5 | (bf(0.5) << 16)           # stale slot beyond the count: ignored
    rec[1, 2, 0] = bf(0.5)
    d = decompress_actions(rec.to(torch.int32), P).float().view(2, R, P)
    b = lambda x: float(torch.tensor(x, dtype=torch.bfloat16))
    assert d[0, 0, 0] == 0.0625 and torch.all(d[0, 0, 1:] == b(0.05))
    want = torch.zeros(P)
    want[3], want[17] = 0.25, 0.75
    assert torch.equal(d[0, 1], want)
    assert torch.all(d[1, 2] == 0.5) and torch.all(d[1, :2] == 0)


def test_sparse_fwd_splits_fill_whole_rounds():
    """The forward's row-block split count: within [1, min(R, max, 64)], and ceil(B / 256) x S workgroups fill
    at least 95 % of whole 256-CU rounds when such an S exists (B = 25,600: 100 row blocks -> S = 5, 500 of
    512 slots)."""
    from gsc_amd.agents.native_update import sparse_fwd_splits
    assert sparse_fwd_splits(25600, 1800, 64) == 5
    for B, R, mx in [(25600, 1800, 64), (8192, 1800, 64), (4096, 250, 16), (512, 3, 64), (300, 1, 8)]:
        S = sparse_fwd_splits(B, R, mx)
        assert 1 <= S <= max(1, min(R, mx, 64))
        wgs = -(-B // 256) * S
        rounds = -(-wgs // 256)
        if rounds >= 2 and wgs / (rounds * 256) < 0.95:   # no S reaches 95 %: the best one is taken
            best = max(-(-B // 256) * s / (max(2, -(-(-(-B // 256) * s) // 256)) * 256)
                       for s in range(1, max(1, min(R, mx, 64)) + 1))
            assert abs(wgs / (max(2, rounds) * 256) - best) < 1e-9


def test_replay_plan_per_config():
    """Ring representation and capacity of the three headline configs on a 288 GB MI355X (E = 256 envs,
    mem_limit 10,000 -> 2M requested): Abilene and syn50 dense at full capacity, syn200 sparse at full capacity
    (the dense ring would hold ~107k); forcing and disabling; no HBM -> dense within 4 GB."""
    from gsc_amd.agents.ddpg import replay_plan
    hbm = 288e9
    cases = {"abilene": (24, 3, 24 * 3 * 24), "syn50": (50, 3, 50 * 9 * 50), "syn200": (200, 3, 200 * 9 * 200)}
    for name, (P, F, A) in cases.items():
        sparse, per, budget = replay_plan(2_000_000, P, F, A, 2, hbm, True)
        assert sparse == (name == "syn200"), name
        assert min(2_000_000, budget // per) == 2_000_000, name
    sparse, per, budget = replay_plan(2_000_000, 200, 3, 360_000, 2, hbm, True, mode="0")
    assert not sparse and budget // per < 250_000   # dense syn200 rows: ~238k transitions in 60 % of HBM
    assert replay_plan(2_000_000, 24, 3, 1728, 2, hbm, True, mode="1")[0]
    assert not replay_plan(2_000_000, 200, 3, 360_000, 2, hbm, False, mode="1")[0]
    assert replay_plan(2_000_000, 200, 3, 360_000, 2, 0, True)[0] is False
