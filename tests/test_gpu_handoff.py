"""Overlapped trainer (simulator on its CU-masked stream, act path on its own stream): the act <-> simulator
hand-off by sequence words (signal / wait kernels, the default) gives bit-identical training to the event
hand-off (GSC_STREAM_VALUES=0) -- the same transitions, metrics and learner parameters."""
import os

import pytest
import torch
import yaml

from tests.conftest import cfg_path

pytestmark = pytest.mark.gpu


def _run(words: str):
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    os.environ["GSC_STREAM_VALUES"] = words
    try:
        cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
        cfg["episode_steps"] = 12
        nets = [cfg_path("networks", "abilene", f) for f in ("abilene-in4-rand-cap1-2.graphml",
                                                             "abilene-in4-rand-cap0-2.graphml")]
        sim = load_batched_from_paths(nets, cfg_path("service_functions", "abc.yaml"),
                                      cfg_path("config", "simulator", "sample_config.yaml"), cfg, 64,
                                      device="cuda", seed=5)
        tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=64, batch_size=512, learning_starts=4, seed=2,
                                                    check_every=0, replay_capacity=256),
                            network_schedule=[0, 1], period=1)  # topology switches at every episode end
        assert tr.sim_stream is not None and tr.act_stream is not None, "overlapped act / simulator streams"
        assert bool(tr._words) == (words == "1")
        for _ in range(30):
            tr.step()
        m = tr.metrics()
        torch.cuda.synchronize()
        n = len(tr.replay)
        return (m["succ"], m["drop"], tr.learner.updates, tr.learner.actor_flat.view().clone(), tr.topo.clone(),
                tr.learner.critic_flat.view().clone(), tr.replay.obs[:n].clone(), tr.replay.rewards[:n].clone())
    finally:
        os.environ.pop("GSC_STREAM_VALUES", None)


def test_word_handoff_matches_event_handoff():
    a, b = _run("1"), _run("0")
    assert a[2] == b[2] >= 20
    assert a[0] == b[0] and a[1] == b[1] and a[0] + a[1] > 0
    assert torch.equal(a[4], b[4]) and int(a[4][0]) == 0  # two switches: back on topology 0
    for x, y in zip(a[3:], b[3:]):
        assert torch.equal(x, y)


def test_handoff_timeout_fails_at_that_step():
    """A simulator signal that never comes: the act's wait times out (0.2 s here), sets the mapped host flag, and
    the trainer raises within its run-ahead bound of that step -- not at the episode end (200 steps)."""
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    sim = load_batched_from_paths([cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")],
                                  cfg_path("service_functions", "abc.yaml"),
                                  cfg_path("config", "simulator", "sample_config.yaml"), cfg, 64, device="cuda", seed=5)
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=64, batch_size=512, learning_starts=2, seed=2, check_every=0,
                                                replay_capacity=256, handoff_timeout_s=0.2))
    if not tr._words:
        pytest.skip("sequence-word hand-off not in use on this device")
    for _ in range(6):
        tr.step()
    nat = tr.sim.native
    real = nat.signal_word
    dropped = []

    def drop_once(stream, word, value):
        if word == tr._words and not dropped:
            dropped.append(tr.global_step)
            return None
        return real(stream, word, value)

    lost = tr.global_step
    tr.sim.native.signal_word = drop_once
    try:
        with pytest.raises(RuntimeError, match="hand-off"):
            for _ in range(60):
                tr.step()
    finally:
        tr.sim.native.signal_word = real
        torch.cuda.synchronize()
    assert dropped == [lost]
    assert tr.global_step - lost <= tr._AHEAD + 3, (lost, tr.global_step)
