"""One large-graph backward at B = 64: launch errors surface, partial rows inspected."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from gsc_amd.coordsim.reader import load_topology  # noqa: E402
from gsc_amd.models import GNNEmbedder, GraphSet  # noqa: E402

gs = GraphSet([load_topology(os.path.join(ROOT, f"configs/networks/synthetic/syn200-in16-cap1-3-s{i}.graphml"))
               for i in range(3)], 200, "cuda")
emb = GNNEmbedder(3, 22, 2, "mean", 2).cuda()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
topo = torch.randint(0, 3, (B,), device="cuda")
x = torch.rand(B, 200, 3, device="cuda") * gs.node_mask[topo].unsqueeze(-1)
out = emb(x, topo, gs, use_native=True)
g = torch.autograd.grad(out.sum(), list(emb.parameters()))
torch.cuda.synchronize()
from gsc_amd.ops.gnn import _PARTIALS  # noqa: E402
for k, p in _PARTIALS.items():
    rows = min(B, 256)
    print("partials", p.shape, "nan rows", int(torch.isnan(p[:rows]).any(1).sum()), "of", rows, "first row", p[0, :8].tolist())
print("grad nan", [bool(torch.isnan(t).any()) for t in g])
if os.environ.get("GSC_LG_PROF") == "1":
    from gsc_amd.native import load
    v = load().gnn_lg_prof()
    print("phase cycles", v[16:29])
    print("nonfinite: DY0", v[30], "XL", v[13], "XR", v[14], "DY", v[15], "HT", v[29], "dxr", v[31], "dxl", v[12], "SC", v[6], "DS", v[7])
