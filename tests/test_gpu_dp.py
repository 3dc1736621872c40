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


def test_rccl_world1_dp_path_bit_identical():
    """GSC_DIST_FORCE=1: a world-size-1 RCCL communicator carries every collective of the DP path (the
    gradient all-reduces captured in the one update graph; the fallback's five graphs with eager all-reduces
    between them; ZeRO-1 reduce-scatter / all-gather; bf16 gradient all-reduce); with one rank the DP learner
    equals the process-local learner bit for bit."""
    env = {**os.environ, "GSC_DIST_FORCE": "1", "OMP_NUM_THREADS": "2"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GSC_DIST_BACKEND", "GSC_DP_GRAD_BF16"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "dp_rccl1.py")], capture_output=True,
                         text=True, timeout=110, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    print(res)
    assert res["backend"] == "nccl" and res["world"] == 1 and res["forced"]
    assert res["ref_graphs"] == 1 and res["dp_graphs"] == 1 and res["eager_graphs"] == 5
    assert res["dp_bitwise"] and res["dp_grad_bitwise"] and res["eager_bitwise"], res
    assert res["zero"] and res["zero_max_abs_diff"] < 1e-6, res
    assert res["bf16"] and res["bf16_max_abs_diff"] < 4 * 1e-3, res


def test_rccl_world1_bench_check_replicas():
    """bench.py's --check-replicas over the forced world-size-1 RCCL group, with the simulator on its
    CU-masked stream and the learner's collectives captured in its update graph."""
    env = {**os.environ, "GSC_DIST_FORCE": "1"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GSC_DIST_BACKEND"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "4",
                          "--envs", "64", "--check-replicas"], capture_output=True, text=True, timeout=110, cwd=ROOT,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    chk = [l for l in lines if "replicas_identical" in l][0]
    rec = [l for l in lines if "metric" in l][0]
    assert chk["replicas_identical"] and chk["graphed"] and chk["updates"] >= 9
    assert rec["config"]["dist_forced"] and rec["n_gpus"] == 1 and rec["value"] > 0
