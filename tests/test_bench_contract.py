"""bench.py output contract: one JSON line with the driver's keys (CPU run, tiny sizes)."""
import json
import os
import subprocess
import sys

from tests.conftest import ROOT

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", *args], capture_output=True,
                       text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_json_contract():
    rec = _run("--envs", "4", "--steps", "2", "--warmup", "1")
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["metric"].startswith("env-steps/sec (whole node)")
    assert abs(rec["value"] - 4 * 2 / (rec["ms_per_step"] * 2 / 1e3)) / rec["value"] < 0.01
    assert rec["vs_baseline"] == round(rec["value"] / 57.4, 1)
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in rec["config"]
    assert rec["config"]["parallelism"] == "dp1" and rec["config"]["global_batch"] == 400
    assert 0.0 <= rec["success_ratio"] <= 1.0


def test_bench_json_contract_two_ranks_gloo():
    """The driver's N>1 launch (torch.distributed.run, one rank per device) on CPU/gloo: one JSON line from
    rank 0, whole-job value over both ranks, dp2, and bit-identical parameter replicas after the timed steps."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--device", "cpu", "--envs", "4", "--steps", "2", "--warmup", "1",
                        "--check-replicas"], capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    recs = [l for l in lines if "metric" in l]
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert abs(rec["value"] - 2 * 4 * 2 / (rec["ms_per_step"] * 2 / 1e3)) / rec["value"] < 0.01
    assert any(l.get("replicas_identical") is True for l in lines), r.stdout
