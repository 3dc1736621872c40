"""Phase cycles of the large-graph fused GATv2 kernels (GSC_LG_PROF=1 variants; shader-clock cycles per graph,
summed over the workgroup's barriers as seen by thread 0): where a 200-node graph's time goes."""
import os
import sys

os.environ["GSC_LG_PROF"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from gsc_amd.coordsim.reader import load_topology  # noqa: E402
from gsc_amd.models import GNNEmbedder, GraphSet  # noqa: E402
from gsc_amd.native import load  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 25600
gs = GraphSet([load_topology(os.path.join(ROOT, f"configs/networks/synthetic/syn200-in16-cap1-3-s{i}.graphml"))
               for i in range(3)], 200, "cuda")
emb = GNNEmbedder(3, 22, 2, "mean", 2).cuda()
topo = torch.randint(0, 3, (B,), device="cuda")
x = torch.rand(B, 200, 3, device="cuda") * gs.node_mask[topo].unsqueeze(-1)
nat = load()
with torch.no_grad():
    emb(x, topo, gs, use_native=True)
torch.cuda.synchronize()
nat.gnn_lg_prof()
for _ in range(2):
    with torch.no_grad():
        emb(x, topo, gs, use_native=True)
torch.cuda.synchronize()
f = nat.gnn_lg_prof()
names = ["wait prev graph", "stage topo/x", "node linears", "attention", "store rows", "pool"]
print(f"forward, cycles per graph (B={B}, 2 runs): total {sum(f[:6]) / (2 * B):.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:18s} {f[k] / (2 * B):9.0f}")
out = emb(x, topo, gs, use_native=True)
g = torch.autograd.grad(out.sum(), list(emb.parameters()))
torch.cuda.synchronize()
nat.gnn_lg_prof()
out = emb(x, topo, gs, use_native=True)
g = torch.autograd.grad(out.sum(), list(emb.parameters()))
torch.cuda.synchronize()
v = nat.gnn_lg_prof()
b = v[16:29]
names = ["wait prev graph", "stage topo/x/dY", "rc node linears", "rc attention", "rc store rows", "x image again",
         "linears + HT", "targets (step 2)", "sources (step 3)", "DT / DN images", "MFMA dW / dX", "dY rows",
         "block-0 flush"]
print(f"backward, cycles per graph: total {sum(b) / B:.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:18s} {b[k] / B:9.0f}")
