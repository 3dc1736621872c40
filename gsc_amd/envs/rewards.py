"""Reward objectives (reference: ``src/rlsp/envs/gym_env.py:223-380``).

Supported objectives: ``prio-flow`` (optional EWMA ``auto`` target),
``soft-deadline``, ``soft-deadline-exp`` and ``weighted``.  The component
rewards are computed from the last run window's statistics.
"""
from __future__ import annotations

import numpy as np

SUPPORTED_OBJECTIVES = {"prio-flow", "soft-deadline", "soft-deadline-exp", "weighted"}


def flow_reward(succ, drop):
    """``(success ratio, (succ - drop) / (succ + drop))``; both 0 when no flow finished."""
    if succ + drop > 0:
        return succ / (succ + drop), (succ - drop) / (succ + drop)
    return 0, 0


def delay_reward(avg_delay, succ_ratio, min_delay, diameter):
    delay = max(avg_delay, min_delay)
    if succ_ratio == 0:
        return delay, -1
    return delay, float(np.clip(((min_delay - delay) / diameter) + 1, -1, 1))


class RewardCalculator:
    """Stateful (EWMA) reward computation shared by the scalar and batched envs."""

    def __init__(self, agent_config: dict, sf_list: dict, network_diameter: float = 15.0):
        self.cfg = agent_config
        self.objective = agent_config["objective"]
        if self.objective not in SUPPORTED_OBJECTIVES:
            raise ValueError(f"Unexpected objective {self.objective}. Must be in {SUPPORTED_OBJECTIVES}.")
        self.target_success = agent_config.get("target_success")
        self.soft_deadline = agent_config.get("soft_deadline")
        self.network_diameter = network_diameter
        self.sf_list = sf_list
        vnf_delays = sum(sf["processing_delay_mean"] for sf in sf_list.values())
        self.min_delay = vnf_delays
        self.max_delay = vnf_delays + len(sf_list) * network_diameter
        self.ewma_flows = 1.0

    def update_ewma(self, value, weight=0.5):
        self.ewma_flows = weight * value + (1 - weight) * self.ewma_flows

    def node_reward_shaped(self, num_nodes, placement) -> float:
        num_sfs = len(self.sf_list)
        used = 0.0
        for sfs in placement.values():
            if len(sfs) > 0:
                used += ((len(sfs) - 1) / (num_sfs - 1)) * 0.5 + 0.5 if num_sfs > 1 else 1.0
        return 2 * (-used / num_nodes) + 1

    def instance_reward(self, num_nodes, placement) -> float:
        num_sfs = len(self.sf_list)
        n_inst = sum(len(v) for v in placement.values())
        return 2 * (-n_inst / (num_nodes * num_sfs)) + 1

    def __call__(self, succ, drop, avg_delay, num_nodes, placement) -> float:
        succ_ratio, f_r = flow_reward(succ, drop)
        delay, d_r = delay_reward(avg_delay, succ_ratio, self.min_delay, self.network_diameter)
        n_r = self.node_reward_shaped(num_nodes, placement)
        i_r = self.instance_reward(num_nodes, placement)
        obj = self.objective
        if obj == "prio-flow":
            n_r = i_r = 0
            target = self.target_success
            if target == "auto":
                target = 0.9 * self.ewma_flows
                self.update_ewma(succ_ratio)
            if succ_ratio < target:
                d_r = -1
        elif obj == "soft-deadline":
            n_r = i_r = 0
            if delay > self.soft_deadline:
                f_r = -1
            else:
                d_r = float(np.clip(-self.soft_deadline / self.network_diameter, -1, 1))
        elif obj == "soft-deadline-exp":
            f_r = n_r = i_r = 0
            util = 1.0
            if delay > self.soft_deadline:
                util = float(np.clip(-np.log10((1 / self.cfg["dropoff"]) * (delay - self.soft_deadline)), 0, 1))
            d_r = succ_ratio * util
        else:  # weighted
            f_r *= self.cfg.get("flow_weight", 0)
            d_r *= self.cfg.get("delay_weight", 0)
            n_r *= self.cfg.get("node_weight", 0)
            i_r *= self.cfg.get("instance_weight", 0)
        total = f_r + d_r + n_r + i_r
        assert -4 <= total <= 4, f"Unexpected total reward: {total}."
        return float(total)
