"""CLI / experiment layout / checkpoint-resume / inference (CPU, tiny episodes).

Result layout follows the reference (src/rlsp/agents/main.py:166-235, main.py:47-50);
``trained_actor.pt``/``checkpoint.pt`` load with ``weights_only=True`` and ``agent_helper.obj`` is
JSON.  Resume must be exact: train k episodes, checkpoint, train m more == train k+m straight.
"""
import json
import os

import pytest
import torch
import yaml
from click.testing import CliRunner

from tests.conftest import ROOT, cfg_path

NET = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
SVC = cfg_path("service_functions", "abc.yaml")
SIM = cfg_path("config", "simulator", "sample_config.yaml")
FILES = ("trained_actor.pt", "checkpoint.pt", "agent_helper.obj", "rewards.csv", "metrics.jsonl", "input.yaml",
         "training.log", "result.yaml", "test_result.yaml", "placements.csv", "metrics.csv", "drop_reasons.csv",
         "run_flows.csv", "runtimes.csv", "node_metrics.csv", "rl_state.csv", "abc.yaml", "sample_config.yaml")


@pytest.fixture()
def small(tmp_path, monkeypatch):
    monkeypatch.chdir(ROOT)
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    cfg.update(episode_steps=4, nb_steps_warmup_critic=3, mem_limit=64, actor_hidden_layer_nodes=[32],
               critic_hidden_layer_nodes=[16])
    agent = tmp_path / "agent.yaml"
    agent.write_text(yaml.safe_dump(cfg))
    sched = tmp_path / "scheduler.yaml"
    sched.write_text(yaml.safe_dump({"training_network_files": [NET], "inference_network": NET, "period": 10}))
    return tmp_path, str(agent), str(sched)


def _run(args):
    from main import cli
    res = CliRunner().invoke(cli, args, catch_exceptions=False)
    assert res.exit_code == 0, res.output
    return res.output


def _runs(root):
    base = os.path.join(root, "agent", "scheduler", "abc", "sample_config")
    return base, sorted(os.listdir(base))


@pytest.mark.parametrize("backend", ["oracle", "batched"])
def test_cli_train_test_layout(small, backend):
    tmp, agent, sched = small
    out = _run([agent, NET, SVC, SIM, sched, "2", "--seed", "1234", "--backend", backend, "--envs", "4",
                "--results-root", str(tmp / "results")])
    assert "test on abilene" in out
    base, runs = _runs(tmp / "results")
    assert len(runs) == 1 and runs[0].endswith("_seed1234")
    d = os.path.join(base, runs[0])
    for f in FILES:
        assert os.path.exists(os.path.join(d, f)), f
    assert yaml.safe_load(open(os.path.join(d, "input.yaml"))) == {"num_ingress": 4, "algorithm": "ddpg"} or \
        yaml.safe_load(open(os.path.join(d, "input.yaml")))["num_ingress"] == 4
    rewards = open(os.path.join(d, "rewards.csv")).read().split()
    assert len(rewards) == 2  # header-less, one row per (lockstep) episode
    h = json.load(open(os.path.join(d, "agent_helper.obj")))
    assert h["seed"] == 1234 and h["episode_steps"] == 4
    from gsc_amd.utils.checkpoint import load_actor
    actor, hdr = load_actor(os.path.join(d, "trained_actor.pt"))
    assert hdr["action_dim"] == 1728 and hdr["n_pad"] == 24
    ck = torch.load(os.path.join(d, "checkpoint.pt"), weights_only=True)
    assert ck["state"]["backend"] == backend and ck["state"]["episode"] == 2
    lines = [json.loads(x) for x in open(os.path.join(d, "metrics.jsonl"))]
    assert any("charts/episodic_return" in x for x in lines)
    assert any("charts/success_ratio" in x for x in lines)


def _helper(tmp, agent, sched, seed=7):
    from gsc_amd.utils.experiment import setup
    return setup(agent, NET, SVC, SIM, sched, seed, 3, results_root=str(tmp / f"r{seed}"))


@pytest.mark.parametrize("backend", ["oracle", "batched"])
def test_resume_is_exact(small, backend):
    from gsc_amd.agents import SimpleDDPG
    tmp, agent, sched = small
    kw = dict(backend=backend, num_envs=4, device="cpu", results_writers=False)
    a = SimpleDDPG(_helper(tmp, agent, sched), **kw)
    a.train(2)
    path = str(tmp / "ck.pt")
    a.save_checkpoint(path)
    a.train(1)
    b = SimpleDDPG(_helper(tmp, agent, sched), **kw)
    b.load_checkpoint(path)
    b.train(1)
    assert a.global_step == b.global_step == 12
    assert torch.equal(a.learner.actor_flat.flat, b.learner.actor_flat.flat)
    assert torch.equal(a.learner.critic_flat.flat, b.learner.critic_flat.flat)
    assert torch.equal(a.learner.target_critic_flat.flat, b.learner.target_critic_flat.flat)


def test_test_only_and_best_reproduce(small):
    tmp, agent, sched = small
    root = str(tmp / "results")
    out1 = _run([agent, NET, SVC, SIM, sched, "2", "--seed", "11", "--backend", "oracle", "--results-root", root])
    base, runs = _runs(root)
    out2 = _run([agent, NET, SVC, SIM, sched, "1", "--seed", "11", "--backend", "oracle", "-t", runs[0],
                 "--results-root", root])
    line = lambda o: [x for x in o.splitlines() if x.startswith("test on")][0]
    assert line(out1) == line(out2)
    out3 = _run([agent, NET, SVC, SIM, sched, "1", "--seed", "11", "--backend", "oracle", "-b", "--results-root", root])
    assert line(out3) == line(out1)
    # -w resumes (episode counter continues)
    _run([agent, NET, SVC, SIM, sched, "1", "--seed", "12", "--backend", "oracle", "-w",
          os.path.join(base, runs[0]), "--results-root", root])
    base, runs2 = _runs(root)
    new = [r for r in runs2 if r.endswith("_seed12")][0]
    ck = torch.load(os.path.join(base, new, "checkpoint.pt"), weights_only=True)
    assert ck["state"]["episode"] == 3


def test_inference_script(small):
    tmp, agent, sched = small
    root = str(tmp / "results")
    _run([agent, NET, SVC, SIM, sched, "1", "--seed", "5", "--backend", "oracle", "--results-root", root])
    base, runs = _runs(root)
    import inference
    r1 = inference.main([os.path.join(base, runs[0])])
    r2 = inference.main([os.path.join(base, runs[0]), "--envs", "2"])
    assert r1[0]["success_ratio"] == pytest.approx(r2[0]["success_ratio"])  # deterministic config


def test_oracle_trains_at_first_episode_end_when_warmup_equals_episode(small):
    """Reference simple_ddpg.py:308 gates the episode-end updates on global_step >= warm-up - 1: with
    nb_steps_warmup_critic == episode_steps the first episode already ends with episode_steps updates."""
    from gsc_amd.agents import SimpleDDPG
    tmp, agent, sched = small
    cfg = yaml.safe_load(open(agent))
    cfg["nb_steps_warmup_critic"] = cfg["episode_steps"]
    open(agent, "w").write(yaml.safe_dump(cfg))
    a = SimpleDDPG(_helper(tmp, agent, sched), backend="oracle", device="cpu", results_writers=False)
    a.train(1)
    assert a.learner.updates == cfg["episode_steps"]
