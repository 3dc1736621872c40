"""Diagnostic: native update (composed / materialised) vs fp32 CPU reference and the bf16 autocast path
with three topologies of different node counts (different action masks)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tests.test_gpu_learner import _batch, _cfg, _learners, _per_param_err  # noqa: E402

T = 3
cfg = _cfg()
ref, comp = _learners(cfg, T)
os.environ["GSC_COMPOSE"] = "0"
_, mat = _learners(cfg, T)
mat.native_update(512)          # built lazily: decide the path while the variable is set
os.environ["GSC_COMPOSE"] = "1"
_, auto = _learners(cfg, T)
auto.native_ok = False
print("compose flags:", comp.native_update(512).compose, mat.native_update(512).compose)
for k in range(3):
    bc, bg = _batch(512, T, "cpu", seed=11 + k), _batch(512, T, "cuda", seed=11 + k)
    ref.update(bc)
    for l in (comp, mat, auto):
        l.update(bg)
    torch.cuda.synchronize()
    print(k, {key: [round(float(l.last[key]), 5) for l in (ref, comp, mat, auto)] for key in ("qf1_loss", "actor_loss", "qf1_values")})
    if k == 0:
        for nm in ("critic_flat", "actor_flat"):
            fm, fc = getattr(mat, nm), getattr(comp, nm)
            e = {n: float((fm.grad[o:o + p.numel()] - fc.grad[o:o + p.numel()]).norm()
                          / fm.grad[o:o + p.numel()].norm().clamp_min(1e-12))
                 for n, p, o in zip(fm.names, fm.params, fm.offsets)}
            print(f"  {nm} composed vs materialised (native):", {n: round(v, 4) for n, v in e.items()})
            e = [_per_param_err(getattr(ref, nm), getattr(l, nm)) for l in (comp, mat, auto)]
            for n in e[0]:
                print(f"  {nm} {n}: comp {e[0][n]:.4f} mat {e[1][n]:.4f} auto {e[2][n]:.4f}")

# critic frozen (lr 0): the actor gradient of the first update goes through the same critic in every
# implementation, so its error is the function's own rounding, not the chaotic first critic step
ref, gpu = _learners(cfg, T)
_, auto = _learners(cfg, T)
auto.native_ok = False
for l in (ref, gpu, auto):
    l.critic_opt.lr = 0.0
bc, bg = _batch(512, T, "cpu", seed=11), _batch(512, T, "cuda", seed=11)
ref.update(bc)
gpu.update(bg)
auto.update(bg)
torch.cuda.synchronize()
e_n, e_a = _per_param_err(ref.actor_flat, gpu.actor_flat), _per_param_err(ref.actor_flat, auto.actor_flat)
print("frozen critic, actor grads vs fp32:")
for n in e_n:
    print(f"  {n}: native {e_n[n]:.4f} autocast {e_a[n]:.4f}")
