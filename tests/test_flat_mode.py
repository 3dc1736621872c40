"""Flat (non-graph) mode and BASELINE config 1 (4-node line + 1 SFC, one CPU env, 2-layer MLP).

Reference ``models.py:115-122, 151`` sizes the flat actor's first layer for obs + action but feeds
only the observation (Q13: shape error on the first forward); the flat mode here is the evident
intent (actor MLP(flatten(obs)), critic MLP([flatten(obs) | action]))."""
import os

import pytest
import torch
import yaml

from tests.conftest import ROOT, cfg_path

LINE4 = cfg_path("networks", "line", "line4-in1-cap1-delay10.graphml")


def _cfg():
    return yaml.safe_load(open(cfg_path("config", "agent", "sample_agent_flat.yaml")))


def test_flat_models_shapes_and_mask():
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import Actor, GraphSet, QNetwork
    cfg = _cfg()
    P, F_, A = 4, 3, 4 * 1 * 3 * 4
    actor, critic = Actor(cfg, F_, A), QNetwork(cfg, F_, A)
    assert actor.embedder is None and not actor.graph_mode
    assert actor.mlp.layers[0].in_features == P * F_ and critic.mlp.layers[0].in_features == P * F_ + A
    assert [l.out_features for l in actor.mlp.layers] == [64, 64, A]
    g = GraphSet([load_topology(LINE4)], P, "cpu")
    masks = g.action_masks(1, 3)
    x, topo = torch.rand(5, P, F_), torch.zeros(5, dtype=torch.int64)
    a = actor(x, topo, g, masks)
    assert a.shape == (5, A)
    q = critic(x, topo, g, masks, a)
    assert q.shape == (5, 1)
    # flat critic == its unfolded MLP on [flatten(obs) | action]
    ref = critic.mlp.forward_full(torch.cat([x.reshape(5, -1), a], 1))
    torch.testing.assert_close(q, ref)


def test_flat_oracle_training_runs(tmp_path, monkeypatch):
    monkeypatch.chdir(ROOT)
    from gsc_amd.agents import SimpleDDPG
    from gsc_amd.utils.experiment import setup
    cfg = _cfg()
    cfg.update(episode_steps=20, nb_steps_warmup_critic=10)
    agent = tmp_path / "agent.yaml"
    agent.write_text(yaml.safe_dump(cfg))
    sched = tmp_path / "sched.yaml"
    sched.write_text(yaml.safe_dump({"training_network_files": [LINE4], "inference_network": LINE4, "period": 10}))
    h = setup(str(agent), LINE4, cfg_path("service_functions", "abc.yaml"),
              cfg_path("config", "simulator", "sample_config.yaml"), str(sched), 3, 2,
              results_root=str(tmp_path / "r"))
    a = SimpleDDPG(h, backend="oracle", device="cpu", results_writers=False)
    out = a.train(2)
    assert out["steps"] == 40 and a.learner.updates == 40   # episode-end updates from step 19 on
    r = a.test(episode_steps=5)
    assert 0.0 <= r["success_ratio"] <= 1.0


def test_bench_line_preset_cpu():
    import json
    import subprocess
    import sys
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--preset", "line", "--steps", "5",
                          "--warmup", "2"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["config"]["device"] == "cpu" and rec["config"]["total_envs"] == 1 and rec["value"] > 0
