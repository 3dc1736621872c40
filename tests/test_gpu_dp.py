"""GPU data parallelism rehearsed on one GPU: 2 ranks with gloo collectives through the HIP-graph
learner path and the batched trainer (scripts/dp_rehearsal.py, launched by torch.distributed.run as
a child process).  Checks bit-identical replicas across ranks and agreement with one process
updating on the concatenated batch."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_graphed_dp():
    env = {**os.environ, "GSC_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "2"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "scripts", "dp_rehearsal.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    print(res)
    assert res["world"] == 2 and res["backend"] == "gloo" and res["graphed"]
    assert res["replicas_bitwise"] and res["trainer_replicas_bitwise"]
    assert res["grad_vs_single"] < 1e-3 and res["grad_vs_single_graphed"] < 1e-3, res
    assert res["param_mismatch_frac"] < 1e-3, res
    assert res["trainer_graphed"] and res["trainer_updates"] >= 4 and res["envs_differ"]
    # sharded optimizer (ZeRO-1) on the native kernels
    assert res["zero"] and res["zero_replicas_bitwise"] and res["zero_moment_frac"] == 0.5
    assert res["zero_param_mismatch_frac"] < 1e-3, res
