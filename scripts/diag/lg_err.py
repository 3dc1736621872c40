"""Per-gradient relative error of the large-graph fused GATv2 kernels vs the layer-wise kernels (both against the
fp32 reference) over hidden widths: tells a kernel bug from bf16 operand noise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from gsc_amd.coordsim.reader import load_topology  # noqa: E402
from gsc_amd.models import GNNEmbedder, GraphSet  # noqa: E402

SYN = [os.path.join(ROOT, f"configs/networks/synthetic/syn200-in16-cap1-3-s{i}.graphml") for i in range(3)]


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def run(hidden, lg, iters=2, B=300, seed=0):
    os.environ["GSC_GNN_LG"] = lg
    gs = GraphSet([load_topology(p) for p in SYN], 200, "cuda")
    torch.manual_seed(seed)
    emb = GNNEmbedder(3, hidden, 2, "mean", iters).cuda()
    topo = torch.randint(0, 3, (B,), device="cuda")
    x = torch.rand(B, 200, 3, device="cuda") * gs.node_mask[topo].unsqueeze(-1)
    ps = list(emb.parameters())
    ref = emb.forward_reference(x, topo, gs)
    w = torch.linspace(-1, 1, hidden, device="cuda")
    gref = torch.autograd.grad((ref * w).sum(), ps)
    out = emb(x, topo, gs, use_native=True)
    g = torch.autograd.grad((out * w).sum(), ps)
    return [round(rel(out.detach(), ref.detach()), 4)] + [round(rel(a, b), 4) for a, b in zip(g, gref)]


LG = os.environ.get("LG_MODES", "1,0").split(",")
ITERS = [int(v) for v in os.environ.get("LG_ITERS", "2").split(",")]
for h in [int(v) for v in (sys.argv[1:] or ["8", "12", "16", "22"])]:
    for it in ITERS:
        for lg in LG:
            print(f"H={h} iters={it} lg={lg}", run(h, lg, iters=it), flush=True)
