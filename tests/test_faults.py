"""Fault injection: corrupted gradients are skipped, a dead rank is detected.

* A non-finite gradient (e.g. a corrupted all-reduce bucket) makes the fused Adam/Polyak step a
  no-op for that network (device-side flag, no host sync) and is counted.
* When a data-parallel peer dies, the surviving rank's next collective fails within the process
  group timeout instead of hanging; training can then restart from ``checkpoint.pt``
  (``tests/test_cli.py::test_resume_is_exact``).
"""
import os
import socket
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

from gsc_amd.ops import FlatParams, FusedAdamPolyak


def _opt(dev):
    lin = torch.nn.Linear(8, 4).to(dev)
    fp = FlatParams(lin)
    tgt = FlatParams(torch.nn.Linear(8, 4).to(dev))
    return fp, tgt, FusedAdamPolyak(fp, lr=1e-2, target=tgt, tau=0.5)


def _check_guard(dev):
    fp, tgt, opt = _opt(dev)
    fp.grad.normal_()
    opt.step()
    assert opt.step_count == 1 and opt.skipped_steps == 0
    p0, t0, m0 = fp.flat.clone(), tgt.flat.clone(), opt.m.clone()
    fp.grad[3] = float("nan")
    opt.step()
    assert torch.equal(fp.flat, p0) and torch.equal(tgt.flat, t0) and torch.equal(opt.m, m0)
    assert opt.skipped_steps == 1 and opt.step_count == 1
    fp.grad[3] = 0.0
    fp.grad[5] = float("inf")
    opt.step()
    assert opt.skipped_steps == 2
    fp.grad.normal_()
    opt.step()
    assert opt.step_count == 2 and not torch.equal(fp.flat, p0)


def test_nonfinite_gradient_guard_cpu():
    _check_guard("cpu")


@pytest.mark.gpu
def test_nonfinite_gradient_guard_gpu():
    _check_guard("cuda")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from gsc_amd.parallel.dist import allreduce_sum_, init_distributed
    init_distributed("cpu", timeout_s=20)
    t = torch.ones(4)
    allreduce_sum_(t)                      # one healthy collective
    if rank == 1:
        os._exit(3)                        # injected failure: the peer dies without shutdown
    t0 = time.time()
    try:
        allreduce_sum_(t)
        msg = "no-error"
    except Exception as e:                 # noqa: BLE001 - any collective failure counts as detected
        msg = f"detected {type(e).__name__} after {time.time() - t0:.1f}s"
    with open(out, "w") as f:
        f.write(msg)
    os._exit(0)


def test_dead_rank_is_detected():
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r0.txt")
        port = _free_port()
        ps = [ctx.Process(target=_rank, args=(r, port, out)) for r in range(2)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
        for p in ps:
            if p.is_alive():
                p.kill()
        assert ps[1].exitcode == 3
        msg = open(out).read()
    assert msg.startswith("detected"), msg
