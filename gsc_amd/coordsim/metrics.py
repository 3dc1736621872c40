"""Simulation metrics (reference: ``coordsim/metrics/metrics.py``).

Totals persist over an episode; ``run_*`` entries are reset every
``run_duration`` by the writer process, which defines the window over which
observations and rewards are computed.
"""
from collections import defaultdict
import logging

import numpy as np

log = logging.getLogger(__name__)

DROP_REASONS = ("TTL", "DECISION", "LINK_CAP", "NODE_CAP")


def _d2():
    return defaultdict(float)


def _d3():
    return defaultdict(_d2)


def _i2():
    return defaultdict(int)


def _i3():
    return defaultdict(_i2)


def _i4():
    return defaultdict(_i3)


class Metrics:
    def __init__(self, network, sfs):
        self.metrics = {}
        self.network = network
        self.sfs = sfs
        self.reset_metrics()

    def reset_metrics(self):
        m = self.metrics
        m["generated_flows"] = 0
        m["processed_flows"] = 0
        m["dropped_flows"] = 0
        m["total_active_flows"] = 0
        m["dropped_flows_locs"] = {v: {sf: 0 for sf in list(self.sfs.keys()) + ["EG"]} for v in self.network.nodes}
        m["dropped_flow_reasons"] = {r: 0 for r in DROP_REASONS}
        m["total_processing_delay"] = 0.0
        m["num_processing_delays"] = 0
        m["avg_processing_delay"] = 0.0
        m["total_path_delay"] = 0.0
        m["num_path_delays"] = 0
        m["avg_path_delay"] = 0.0
        m["total_end2end_delay"] = 0.0
        m["avg_end2end_delay"] = 0.0
        m["avg_total_delay"] = 0.0
        m["running_time"] = 0.0
        m["current_active_flows"] = defaultdict(_i3)
        m["current_traffic"] = defaultdict(_d3)
        self.reset_run_metrics()

    def reset_run_metrics(self):
        m = self.metrics
        m["run_dropped_flows_per_node"] = {v: 0 for v in self.network.nodes}
        m["run_dropped_flows"] = 0
        m["run_end2end_delay"] = 0
        m["run_avg_end2end_delay"] = 0.0
        m["run_max_end2end_delay"] = 0.0
        m["run_total_path_delay"] = 0
        m["run_avg_path_delay"] = 0
        m["run_generated_flows"] = 0
        m["run_in_network_flows"] = 0
        m["run_processed_flows"] = 0
        m["run_max_node_usage"] = defaultdict(float)
        m["run_total_requested_traffic"] = defaultdict(_d3)
        m["run_act_total_requested_traffic"] = defaultdict(_d3)
        m["run_total_requested_traffic_node"] = defaultdict(float)
        m["run_total_processed_traffic"] = defaultdict(_d2)
        m["run_flow_counts"] = defaultdict(_i4)

    # event hooks -------------------------------------------------------------------
    def calc_max_node_usage(self, node_id, usage):
        if usage > self.metrics["run_max_node_usage"][node_id]:
            self.metrics["run_max_node_usage"][node_id] = usage

    def add_requesting_flow(self, flow):
        m = self.metrics
        m["run_total_requested_traffic"][flow.current_node_id][flow.sfc][flow.current_sf] += flow.dr
        m["run_act_total_requested_traffic"][flow.current_node_id][flow.sfc][flow.current_sf] += flow.dr

    def add_active_flow(self, flow, node_id, sf):
        m = self.metrics
        m["current_active_flows"][node_id][flow.sfc][sf] += 1
        m["current_traffic"][node_id][flow.sfc][sf] += flow.dr
        m["run_total_processed_traffic"][node_id][sf] += flow.dr

    def remove_active_flow(self, flow, node_id, sf):
        m = self.metrics
        m["current_active_flows"][node_id][flow.sfc][sf] -= 1
        m["current_traffic"][node_id][flow.sfc][sf] -= flow.dr
        if m["current_active_flows"][node_id][flow.sfc][sf] < 0 or m["total_active_flows"] < 0:
            log.critical("negative active flow count")

    def generated_flow(self, flow, node):
        m = self.metrics
        m["generated_flows"] += 1
        m["run_generated_flows"] += 1
        m["total_active_flows"] += 1
        m["run_total_requested_traffic_node"][node] += flow.dr

    def completed_flow(self):
        m = self.metrics
        m["processed_flows"] += 1
        m["run_processed_flows"] += 1
        m["total_active_flows"] -= 1
        assert m["total_active_flows"] >= 0

    def dropped_flow(self, flow, reason):
        m = self.metrics
        assert reason in m["dropped_flow_reasons"]
        flow.dropped = True
        m["dropped_flows"] += 1
        m["total_active_flows"] -= 1
        sf = "EG" if flow.current_sf is None else flow.current_sf
        m["dropped_flows_locs"][flow.current_node_id][sf] += 1
        m["run_dropped_flows_per_node"][flow.current_node_id] += 1
        m["run_dropped_flows"] += 1
        assert m["total_active_flows"] >= 0
        if flow.ttl <= 0:
            reason = "TTL"
        m["dropped_flow_reasons"][reason] += 1

    def add_processing_delay(self, delay):
        self.metrics["num_processing_delays"] += 1
        self.metrics["total_processing_delay"] += delay

    def add_path_delay(self, delay):
        m = self.metrics
        m["num_path_delays"] += 1
        m["total_path_delay"] += delay
        m["run_total_path_delay"] += delay
        if m["run_generated_flows"] > 0:
            m["run_avg_path_delay"] = m["run_total_path_delay"] / m["run_generated_flows"]

    def add_end2end_delay(self, delay):
        m = self.metrics
        m["total_end2end_delay"] += delay
        m["run_end2end_delay"] += delay
        if delay > m["run_max_end2end_delay"]:
            m["run_max_end2end_delay"] = delay

    def running_time(self, start, end):
        self.metrics["running_time"] = end - start

    def get_active_flows(self):
        return self.metrics["current_active_flows"]

    def get_metrics(self):
        m = self.metrics
        m["avg_processing_delay"] = (m["total_processing_delay"] / m["num_processing_delays"]
                                     if m["num_processing_delays"] > 0 else 0)
        m["avg_path_delay"] = m["total_path_delay"] / m["num_path_delays"] if m["num_path_delays"] > 0 else 0
        m["avg_total_delay"] = float(np.mean([m["avg_path_delay"], m["avg_processing_delay"]]))
        m["avg_end2end_delay"] = (m["total_end2end_delay"] / m["processed_flows"]
                                  if m["processed_flows"] > 0 else 0)
        m["run_avg_end2end_delay"] = (m["run_end2end_delay"] / m["run_processed_flows"]
                                      if m["run_processed_flows"] > 0 else 0)
        return m
