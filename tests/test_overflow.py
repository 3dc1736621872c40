"""Simulator pool overflow fails loudly (device flag checked at episode ends and before results)."""
import pytest
import torch
import yaml

from tests.conftest import ROOT, cfg_path


def test_tiny_flow_pool_raises(monkeypatch):
    monkeypatch.chdir(ROOT)
    from gsc_amd.sim.batched import load_batched_from_paths
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    sim = load_batched_from_paths([cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")],
                                  cfg_path("service_functions", "abc.yaml"),
                                  cfg_path("config", "simulator", "sample_config.yaml"), cfg, 2, device="cpu",
                                  caps=dict(flow_cap=2, proc_cap=64, event_cap=256), host_threads=1)
    sim.reset()
    act = torch.full((2, sim.action_dim), 1.0 / 24)
    for _ in range(3):
        sim.step(act)
    with pytest.raises(RuntimeError, match="overflow"):
        sim.check_flags()


def test_trainer_checks_flags_at_episode_end(monkeypatch):
    monkeypatch.chdir(ROOT)
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    cfg.update(episode_steps=3, actor_hidden_layer_nodes=[16], critic_hidden_layer_nodes=[8])
    sim = load_batched_from_paths([cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")],
                                  cfg_path("service_functions", "abc.yaml"),
                                  cfg_path("config", "simulator", "sample_config.yaml"), cfg, 2, device="cpu",
                                  caps=dict(flow_cap=2, proc_cap=64, event_cap=256), host_threads=1)
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=2, batch_size=4, learning_starts=1, check_every=0))
    with pytest.raises(RuntimeError, match="overflow"):
        for _ in range(3):
            tr.step()
