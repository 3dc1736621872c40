"""GPU replay kernels == host path (same Philox index stream, same cursor semantics)."""
import pytest
import torch

from gsc_amd.agents.replay import DeviceReplay

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("A,align", [(1728, 1), (22500, 8)])
def test_device_replay_matches_host(A, align):
    torch.manual_seed(0)
    E, cap = 96, 500
    rs = [DeviceReplay(cap, 24, 3, A, d, action_dtype=torch.bfloat16, seed=42, action_row_align=align)
          for d in ("cpu", "cuda")]
    for step in range(7):
        obs, nxt = torch.rand(E, 24, 3), torch.rand(E, 24, 3)
        act, rew = torch.rand(E, A), torch.randn(E)
        topo = torch.randint(0, 3, (E,))
        done = (torch.rand(E) < 0.2).to(torch.uint8)
        for r in rs:
            d = r.device
            r.add(obs.to(d), topo.to(d), act.to(d), rew.to(d), nxt.to(d), done.to(d))
        t32 = [torch.zeros(3000, dtype=torch.int32, device=r.device) for r in rs]
        bs = [r.sample(3000, topo32=t) for r, t in zip(rs, t32)]
        torch.cuda.synchronize()
        assert torch.equal(t32[1].cpu(), bs[1].topo.cpu().to(torch.int32))
        assert torch.equal(t32[0], bs[0].topo.to(torch.int32))
        assert torch.equal(rs[0].last_indices(3000), rs[1].last_indices(3000).cpu())
        for a, b in zip(*bs):
            assert torch.equal(a, b.cpu())
    assert rs[1].full and torch.equal(rs[1].state.cpu(), rs[0].state)
