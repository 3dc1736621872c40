"""Replay ring (reference src/rlsp/agents/buffer.py:23-89): native insert / Philox sampling.

The index stream is pinned against a pure-Python Philox4x32-10; the GPU kernels draw the same
stream (tests/test_gpu_replay.py)."""
import numpy as np
import pytest
import torch

from gsc_amd.agents.replay import DeviceReplay

M32 = 0xffffffff


def philox4x32_10(k0, k1, ctr):
    c = [ctr & M32, (ctr >> 32) & M32, 0x9E3779B9, 0x243F6A88]
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c[3] ^ k1) & M32, p0 & M32]
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c


def ref_index(seed, draw, b, pos, full, cap):
    u = philox4x32_10(seed, 0x7265706C, (draw << 32) | (b >> 2))[b & 3]
    if full:
        return (pos + 1 + ((u * (cap - 1)) >> 32)) % cap
    return (u * pos) >> 32


def _fill(r, n, E=5):
    for i in range(n):
        v = torch.full((E,), float(i))
        r.add(torch.full((E, 4, 2), float(i)), torch.arange(E) % 2, torch.full((E, 8), float(i)), v,
              torch.full((E, 4, 2), float(i) + 0.5), torch.ones(E, dtype=torch.uint8))


@pytest.mark.parametrize("rounds", [1, 3, 7])
def test_index_stream_matches_python_philox(rounds):
    cap = 20
    r = DeviceReplay(cap, 4, 2, 8, "cpu", seed=1234)
    _fill(r, rounds)
    for draw in range(3):
        b = r.sample(37)
        idx = r.last_indices(37).tolist()
        exp = [ref_index(1234, draw, i, r.pos, r.full, cap) for i in range(37)]
        assert idx == exp
        # gathered rows are the ring rows at those indices
        assert torch.equal(b.obs, r.obs[exp]) and torch.equal(b.actions, r.actions[exp])
        assert torch.equal(b.dones, torch.ones(37))


def test_sampling_excludes_write_cursor_when_full():
    cap = 16
    r = DeviceReplay(cap, 4, 2, 8, "cpu", seed=7)
    _fill(r, 5, E=5)          # 25 rows into 16: full, cursor at 9
    assert r.full and r.pos == 9
    seen = np.zeros(cap, np.int64)
    for _ in range(200):
        r.sample(64)
        seen += np.bincount(r.last_indices(64).numpy(), minlength=cap)
    assert seen[r.pos] == 0
    assert (np.delete(seen, r.pos) > 0).all()
    # roughly uniform over the other 15 rows
    f = np.delete(seen, r.pos) / seen.sum()
    assert np.abs(f - 1 / 15).max() < 0.01


def test_insert_wraps_and_converts():
    r = DeviceReplay(6, 4, 2, 8, "cpu", action_dtype=torch.bfloat16, seed=0)
    _fill(r, 2, E=4)          # rows 0..3 <- 0, rows 4,5,0,1 <- 1
    assert r.pos == 2 and r.full
    assert r.rewards.tolist() == [1, 1, 0, 0, 1, 1]
    assert r.actions.dtype == torch.bfloat16 and float(r.actions[2, 0]) == 0.0 and float(r.actions[0, 0]) == 1.0
    assert r.topo.tolist() == [0, 1, 0, 1, 0, 1]
    assert torch.equal(r.state[:2], torch.tensor([2, 1]))


def test_rng_state_roundtrip():
    r = DeviceReplay(20, 4, 2, 8, "cpu", seed=99)
    _fill(r, 2)
    r.sample(10)
    st = r.rng_state()
    a = r.sample(10).obs.clone()
    q = DeviceReplay(20, 4, 2, 8, "cpu", seed=0)
    _fill(q, 2)
    q.set_rng_state(st)
    assert torch.equal(q.sample(10).obs, a)


def test_fused_sample_writes_int32_topology_ids():
    r = DeviceReplay(50, 4, 3, 6, "cpu", seed=3)
    topo = torch.arange(20) % 5
    r.add(torch.rand(20, 4, 3), topo, torch.rand(20, 6), torch.rand(20), torch.rand(20, 4, 3),
          torch.zeros(20, dtype=torch.uint8))
    t32 = torch.full((64,), -1, dtype=torch.int32)
    b = r.sample(64, topo32=t32)
    assert torch.equal(t32, b.topo.to(torch.int32))
    assert torch.equal(b.topo, topo[r.last_indices(64).long()])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_padded_action_rows(dtype):
    """action_row_align: ring / batch rows padded with zero columns (16-byte aligned bf16 rows for the
    native learner at A % 8 != 0); the first A columns hold the actions, checkpoints keep [.., :A]."""
    A = 13
    r = DeviceReplay(10, 4, 2, A, "cpu", action_dtype=dtype, seed=5, action_row_align=8)
    assert r.actions.shape == (10, 16) and r.action_dim == A
    act = torch.rand(6, A)
    r.add(torch.rand(6, 4, 2), torch.zeros(6, dtype=torch.long), act, torch.rand(6), torch.rand(6, 4, 2),
          torch.zeros(6, dtype=torch.uint8))
    assert torch.equal(r.actions[:6, :A], act.to(dtype)) and not r.actions[:, A:].any()
    b = r.sample(32)
    assert b.actions.shape == (32, 16)
    assert torch.equal(b.actions[:, :A], r.actions[r.last_indices(32).long(), :A]) and not b.actions[:, A:].any()
    sd = r.state_dict()
    assert sd["actions"].shape == (6, A)
    q = DeviceReplay(10, 4, 2, A, "cpu", action_dtype=dtype, seed=5, action_row_align=8)
    q.load_state_dict(sd)
    assert torch.equal(q.actions, r.actions)
