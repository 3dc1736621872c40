"""Gym-style single environment over one simulator (reference: ``src/rlsp/envs/gym_env.py``).

* Network scheduler: the first training reset uses
  ``training_network_files[0]``; every ``period`` episodes a new simulator is
  built on the next file (cyclic); test mode always uses ``inference_network``
  (gym_env.py:103-128).
* ``step`` returns ``(obs, reward, terminated, truncated=False, info)`` with
  ``terminated`` after ``episode_steps`` steps.

Reference quirk Q1 (hard-coded 24 nodes / 37 edges / 15 ms diameter) is kept
as the *default* for model/action-shape compatibility; the agent config keys
``max_nodes``, ``max_edges`` and ``network_diameter`` (``auto`` = from the
topology's APSP) override it.
"""
from __future__ import annotations

import inspect
import logging
import os
from typing import Callable, Optional

import numpy as np
from tqdm import tqdm

from gsc_amd.coordsim.reader import get_sf, get_sfc
from .limits import EnvironmentLimits
from .rewards import RewardCalculator
from .wrapper import SimulatorWrapper

logger = logging.getLogger(__name__)

DEFAULT_MAX_NODES = 24
DEFAULT_MAX_EDGES = 37
DEFAULT_DIAMETER = 15


def make_simulator(network_file, service_file, sim_config_file, test_mode=False, test_dir=None):
    """Factory for the scalar coord-sim backend (reference ``util_functions.create_simulator``)."""
    from gsc_amd.coordsim.simulator import Simulator
    return Simulator(network_file, service_file, sim_config_file, test_mode=test_mode, test_dir=test_dir)


class GymEnv:
    metadata = {"render_modes": ["human"]}

    def __init__(self, agent_config, scheduler_conf, network_file, service_file, seed=None, sim_seed=None,
                 render_mode: str = None, agent_helper=None, sim_config_file: Optional[str] = None,
                 simulator_factory: Optional[Callable] = None, test_mode: Optional[bool] = None):
        self.network_file = network_file
        self.service_file = service_file
        self.agent_config = agent_config
        self.scheduler_conf = scheduler_conf
        self.agent_helper = agent_helper
        self.sim_config_file = sim_config_file or (agent_helper.sim_config_path if agent_helper else None)
        self.simulator_factory = simulator_factory or make_simulator
        self._test_mode = test_mode
        self.simulator = None
        self.current_network = None
        self.sim_seed = sim_seed
        self.simulator_wrapper = None
        self.current_simulator_state = None
        self.render_mode = render_mode
        self.run_count = 0
        self.episode_count = 0
        self.np_random = np.random.default_rng(seed)

        self.sfc_list = get_sfc(service_file)
        self.sf_list = get_sf(service_file)
        diam = agent_config.get("network_diameter", DEFAULT_DIAMETER)
        self._auto_diameter = diam == "auto"
        self.network_diameter = DEFAULT_DIAMETER if self._auto_diameter else float(diam)
        self.env_limits = EnvironmentLimits(
            num_nodes=agent_config.get("max_nodes", DEFAULT_MAX_NODES), sfc_list=self.sfc_list,
            node_obs_space_len=len(agent_config["observation_space"]),
            link_obs_space_len=len(agent_config.get("link_observation_space", [])),
            graph_mode=agent_config["graph_mode"], num_edges=agent_config.get("max_edges", DEFAULT_MAX_EDGES))
        self.rewarder = RewardCalculator(agent_config, self.sf_list, self.network_diameter)
        self.min_delay, self.max_delay = self.rewarder.min_delay, self.rewarder.max_delay
        self.action_space = self.env_limits.action_space
        self.observation_space = self.env_limits.observation_space
        self.permutation = None
        self.objective = agent_config["objective"]

    @property
    def test_mode(self) -> bool:
        if self._test_mode is not None:
            return self._test_mode
        return bool(self.agent_helper is not None and self.agent_helper.test_mode is True)

    def _create_simulator(self, network):
        self.current_network = network
        if self.agent_helper is not None:
            self.agent_helper.network_path = network
            self.agent_helper.result.env_config["network_file"] = network
        test_dir = self.agent_helper.config_dir if self.agent_helper is not None else None
        return self.simulator_factory(network, self.service_file, self.sim_config_file,
                                      test_mode=self.test_mode, test_dir=test_dir)

    def _schedule_network(self):
        sched = self.scheduler_conf
        files = sched["training_network_files"]
        if self.test_mode:
            network = sched["inference_network"]
            tqdm.write(f"current network: {os.path.basename(network)}")
            self.simulator = self._create_simulator(network)
            return self.simulator
        if self.simulator is None:
            # first reset (or the first one after a resume at episode ``episode_count``)
            network = files[(self.episode_count // sched["period"]) % len(files)]
            tqdm.write(f"current network: {os.path.basename(network)}")
            self.simulator = self._create_simulator(network)
        elif self.episode_count % sched["period"] == 0 and self.episode_count > 0:
            network = files[(self.episode_count // sched["period"]) % len(files)]
            tqdm.write(f"current network: {os.path.basename(network)}")
            self.simulator = self._create_simulator(network)
        return self.simulator

    def reset(self, seed: int = None, **kwargs):
        if seed is None:
            seed = int(self.np_random.integers(0, np.iinfo(np.int32).max))
        self.simulator = self._schedule_network()
        self.simulator_wrapper = SimulatorWrapper(self.simulator, self.env_limits, self.agent_config["graph_mode"],
                                                  self.agent_config["observation_space"])
        self.run_count = 0
        obs, self.current_simulator_state = self.simulator_wrapper.init(seed)
        if self._auto_diameter and hasattr(self.simulator, "network"):
            from gsc_amd.coordsim.reader import network_diameter
            self.network_diameter = self.rewarder.network_diameter = float(network_diameter(self.simulator.network))
        if self.agent_config.get("shuffle_nodes", False):
            obs, self.permutation = self.simulator_wrapper.permute_node_order(obs)
        return obs, {}

    def step(self, action: np.ndarray):
        done = False
        self.run_count += 1
        if self.agent_config.get("shuffle_nodes", False):
            action = self.simulator_wrapper.reverse_node_permutation(action, self.permutation)
            self.permutation = None
        obs, self.current_simulator_state = self.simulator_wrapper.apply(action)
        reward = self.calculate_reward(self.current_simulator_state)
        if self.agent_config.get("shuffle_nodes", False):
            obs, self.permutation = self.simulator_wrapper.permute_node_order(obs)
        if self.run_count == self.agent_config["episode_steps"]:
            done = True
            self.run_count = 0
            self.episode_count += 1
        return obs, reward, done, False, {}

    def calculate_reward(self, state) -> float:
        s = state.network_stats
        return self.rewarder(s["run_successful_flows"], s["run_dropped_flows"], s["run_avg_end2end_delay"],
                             len(state.network["nodes"]), state.placement)

    def reward_func_repr(self) -> str:
        return inspect.getsource(RewardCalculator.__call__)

    def render(self, mode="human"):
        assert mode in self.metadata["render_modes"]

    def close(self):
        if self.simulator is not None and hasattr(self.simulator, "writer"):
            self.simulator.writer.close()
