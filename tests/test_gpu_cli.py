"""GPU: the CLI trains with the batched device backend (HIP simulator + fused kernels + graphs)."""
import json
import os

import pytest
import yaml
from click.testing import CliRunner

from tests.conftest import ROOT, cfg_path

pytestmark = pytest.mark.gpu


def test_cli_batched_backend_on_gpu(tmp_path, monkeypatch):
    monkeypatch.chdir(ROOT)
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    cfg.update(episode_steps=6, nb_steps_warmup_critic=2)
    agent = tmp_path / "agent.yaml"
    agent.write_text(yaml.safe_dump(cfg))
    net = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
    from main import cli
    res = CliRunner().invoke(cli, [str(agent), net, cfg_path("service_functions", "abc.yaml"),
                                   cfg_path("config", "simulator", "sample_config.yaml"),
                                   cfg_path("config", "scheduler.yaml"), "3", "--seed", "5", "--backend", "batched",
                                   "--envs", "32", "--results-root", str(tmp_path / "r")], catch_exceptions=False)
    assert res.exit_code == 0, res.output
    run = next((tmp_path / "r").rglob("metrics.jsonl"))
    rows = [json.loads(l) for l in open(run)]
    assert sum("charts/success_ratio" in r for r in rows) == 3
    assert (run.parent / "trained_actor.pt").exists() and (run.parent / "checkpoint.pt").exists()
