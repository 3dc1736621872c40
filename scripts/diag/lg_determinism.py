"""Repeat tests/test_gpu_gnn_lg.py::test_lg_deterministic_and_forward2's gradient comparison N times and print
how many runs were bitwise equal (bisecting a nondeterministic gradient in the large-graph GATv2 backward)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_gpu_gnn_lg import _mixed  # noqa: E402
from gsc_amd.models import GNNEmbedder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
gs = _mixed(200)
torch.manual_seed(3)
emb = GNNEmbedder(3, 22, 2, "mean", 2).to("cuda")
topo = torch.randint(0, gs.num_topologies, (B,), device="cuda")
x = torch.rand(B, 200, 3, device="cuda") * gs.node_mask[topo].unsqueeze(-1)
outs, grads = [], []
for _ in range(n):
    out = emb(x, topo, gs, use_native=True)
    outs.append(out.detach().clone())
    grads.append([g.clone() for g in torch.autograd.grad(out.square().sum(), list(emb.parameters()))])
fwd_eq = sum(torch.equal(outs[0], o) for o in outs[1:])
bwd_eq = sum(all(torch.equal(a, b) for a, b in zip(grads[0], g)) for g in grads[1:])
maxd = max(max(float((a - b).abs().max()) for a, b in zip(grads[0], g)) for g in grads[1:])
print(f"forward equal {fwd_eq}/{n - 1}  gradients equal {bwd_eq}/{n - 1}  max |diff| {maxd:.3e}", flush=True)
