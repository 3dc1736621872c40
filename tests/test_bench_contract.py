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
