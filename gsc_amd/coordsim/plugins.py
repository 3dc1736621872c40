"""coord-sim plugins: flow generators, decision makers, forwarders, processors.

Reference files: ``coordsim/flow_generators/*``, ``coordsim/decision_maker/*``,
``coordsim/forwarders/*``, ``coordsim/flow_processors/*``.  The reference
selects plugins with ``eval(class_name)`` over package auto-imports
(``flowsimulator.py:30-41``); here an explicit registry maps the same config
names to classes (``register_plugin`` adds user plugins).

Every ``yield``/``env.process`` below appears in the same order as in the
reference so that event ids - and therefore the resolution of simultaneous
events - match SimPy exactly.
"""
from __future__ import annotations

import random
from typing import Dict, Tuple

import numpy as np

from .flow import Flow

PLUGINS: Dict[str, type] = {}


def register_plugin(cls):
    PLUGINS[cls.__name__] = cls
    return cls


def get_plugin(name: str, base: type):
    try:
        cls = PLUGINS[name]
    except KeyError:
        raise ValueError(f"unknown plugin class {name!r}; known: {sorted(PLUGINS)}") from None
    if not issubclass(cls, base):
        raise TypeError(f"{name} is not a {base.__name__}")
    return cls


# ----------------------------------------------------------------------------------------------
# Flow generators
# ----------------------------------------------------------------------------------------------
class BaseFlowGenerator:
    def __init__(self, env, params):
        self.env = env
        self.params = params

    def generate_flow(self, flow_id, node_id) -> Tuple[float, Flow]:
        raise NotImplementedError

    def _finish(self, flow_id, node_id, dr, size):
        p = self.params
        sfc = np.random.choice([s for s in p.sfc_list.keys()])
        egress = random.choice(p.eg_nodes) if p.eg_nodes else None
        ttl = random.choice(p.ttl_choices)
        flow = Flow(str(flow_id), sfc, dr, size, self.env.now, current_node_id=node_id, egress_node_id=egress, ttl=ttl)
        p.metrics.generated_flow(flow, node_id)
        return flow


@register_plugin
class DefaultFlowGenerator(BaseFlowGenerator):
    """Deterministic or Poisson arrivals, N(mean, std) rates, fixed or Pareto sizes."""

    def generate_flow(self, flow_id, node_id):
        p = self.params
        if p.deterministic_arrival:
            inter_arr = p.inter_arr_mean[node_id]
        else:
            inter_arr = random.expovariate(1.0 / p.inter_arr_mean[node_id])
        dr, size = self.get_flow_dr_size()
        return inter_arr, self._finish(flow_id, node_id, dr, size)

    def get_flow_dr_size(self):
        p = self.params
        while True:
            dr = np.random.normal(p.flow_dr_mean, p.flow_dr_stdev)
            size = p.flow_size_shape if p.deterministic_size else np.random.pareto(p.flow_size_shape) + 1
            if dr >= 0.0 and size >= 0.0:
                return dr, size


@register_plugin
class ListFlowGenerator(BaseFlowGenerator):
    """Draws (inter-arrival, rate, size) from the per-episode pre-generated lists."""

    def generate_flow(self, flow_id, node_id):
        inter_arr, dr, size = self.params.get_next_flow_data(node_id)
        return inter_arr, self._finish(flow_id, node_id, dr, size)


# ----------------------------------------------------------------------------------------------
# Decision makers
# ----------------------------------------------------------------------------------------------
class BaseDecisionMaker:
    decision_type = "Aggregate"

    def __init__(self, env, params):
        self.env = env
        self.params = params

    def decide_next_node(self, flow: Flow):
        raise NotImplementedError


@register_plugin
class DefaultDecisionMaker(BaseDecisionMaker):
    """Deterministic weighted round robin over the schedule (per-run flow counters)."""

    decision_type = "Aggregate"

    def decide_next_node(self, flow: Flow):
        yield self.env.timeout(0)
        if flow.ttl <= 0:
            return None
        if flow.forward_to_eg:
            if flow.egress_node_id is None:
                flow.egress_node_id = flow.current_node_id
            return flow.egress_node_id
        p = self.params
        sf = p.sfc_list[flow.sfc][flow.current_position]
        flow.current_sf = sf
        p.metrics.add_requesting_flow(flow)
        schedule = p.schedule
        if flow.current_node_id in schedule and flow.sfc in schedule[flow.current_node_id]:
            try:
                local = schedule[flow.current_node_id][flow.sfc][sf]
                dests = list(local.keys())
                probs = list(local.values())
                counts = p.metrics.metrics["run_flow_counts"][flow.current_node_id][flow.sfc][sf]
                total = sum(counts.values())
                ratios = [counts[v] / total for v in dests] if total > 0 else [0 for _ in dests]
                diffs = [probs[i] - ratios[i] if probs[i] > 0 else -1 for i in range(len(dests))]
                nxt = dests[int(np.argmax(diffs))]
                counts[nxt] += 1
                return nxt
            except Exception as ex:  # malformed rule: drop (reference typo Q17 fixed)
                p.logger.warning(f"Flow {flow.flow_id}: scheduling rule at {flow.current_node_id} invalid ({ex}).")
                return None
        p.logger.warning(f"Flow {flow.flow_id}: scheduling rule not found at {flow.current_node_id}. Dropping flow!")
        return None


@register_plugin
class ExternalDecisionMaker(BaseDecisionMaker):
    """Per-flow decisions requested from an external algorithm via ``params.flow_trigger``."""

    decision_type = "PerFlow"

    def decide_next_node(self, flow: Flow):
        if flow.ttl <= 0:
            return None
        if flow.forward_to_eg and flow.current_node_id == flow.egress_node_id:
            return flow.current_node_id
        now = self.env.now
        for entry in list(self.env.queue):
            ev = entry[-1]
            if entry[0] == now and ev.triggered and ev.value is not None:
                yield self.env.timeout(random.random() / 10)
        sf = self.params.sfc_list[flow.sfc][flow.current_position] if not flow.forward_to_eg else "EG"
        flow.current_sf = sf
        self.params.metrics.add_requesting_flow(flow)
        self.params.flow_trigger.succeed(value=flow)
        self.params.flow_trigger = self.env.event()
        return "External"


# ----------------------------------------------------------------------------------------------
# Forwarders
# ----------------------------------------------------------------------------------------------
class BaseFlowForwarder:
    def __init__(self, env, params):
        self.env = env
        self.params = params

    def forward_flow(self, flow: Flow, next_node):
        raise NotImplementedError


@register_plugin
class DefaultFlowForwarder(BaseFlowForwarder):
    """Shortest-path forwarding with per-hop link capacity reservation for ``flow.duration``."""

    def forward_flow(self, flow: Flow, next_node):
        p = self.params
        if next_node is None:
            return False
        sp = p.network.graph["shortest_paths"]
        path_delay = 0
        if flow.current_node_id != next_node:
            path_delay = sp[(flow.current_node_id, next_node)][1]
        if flow.ttl - path_delay <= 0:
            flow.ttl = 0
            return False
        if flow.current_node_id == flow.egress_node_id and flow.forward_to_eg:
            flow.departed = True
            flow.success = True
        if flow.current_node_id == next_node:
            if p.writer is not None:
                p.writer.write_flow_action(p, self.env.now, flow, flow.current_node_id, next_node)
        else:
            path = sp[(flow.current_node_id, next_node)][0]
            for hop in path[1:]:
                if p.writer is not None:
                    p.writer.write_flow_action(p, self.env.now, flow, flow.current_node_id, hop)
                if not self.deduct_link_resources(flow, flow.current_node_id, hop):
                    return False
                p.update_passed_traffic(flow.dr, flow.current_node_id, hop)
                hop_delay = sp[(flow.current_node_id, hop)][1]
                if hop == flow.egress_node_id and flow.forward_to_eg:
                    flow.departed = True
                    flow.success = True
                yield self.env.timeout(hop_delay)
                self.env.process(self.return_link_resources(flow, flow.current_node_id, hop))
                flow.current_node_id = hop
            p.metrics.add_path_delay(path_delay)
            flow.end2end_delay += path_delay
            flow.ttl -= path_delay
        return True

    def deduct_link_resources(self, flow, src, dst):
        edge = self.params.network.edges[(src, dst)]
        if edge["remaining_cap"] - flow.dr >= 0:
            edge["remaining_cap"] -= flow.dr
            return True
        return False

    def return_link_resources(self, flow, src, dst):
        yield self.env.timeout(flow.duration)
        edge = self.params.network.edges[(src, dst)]
        edge["remaining_cap"] += flow.dr
        assert edge["remaining_cap"] <= edge["cap"], "edge remaining cap above capacity"


# ----------------------------------------------------------------------------------------------
# Processors
# ----------------------------------------------------------------------------------------------
class BaseFlowProcessor:
    def __init__(self, env, params):
        self.env = env
        self.params = params

    def process_flow(self, flow: Flow):
        raise NotImplementedError

    def get_demanded_cap(self, dr, node_id, sf):
        total = 0.0
        sf_list = self.params.sf_list
        for sf_i, data in self.params.network.nodes[node_id]["available_sf"].items():
            if sf_i == "EG":
                continue
            if sf_i == sf:
                total += sf_list[sf]["resource_function"](data["load"] + dr)
            else:
                total += sf_list[sf_i]["resource_function"](data["load"])
        return total

    def get_processing_delay(self, flow, sf):
        d = self.params.sf_list[sf]
        delay = np.absolute(np.random.normal(d["processing_delay_mean"], d["processing_delay_stdev"]))
        if flow.ttl - delay <= 0:
            flow.ttl = 0
            return False
        self.params.metrics.add_processing_delay(delay)
        flow.end2end_delay += delay
        flow.ttl -= delay
        return delay

    def request_resources(self, flow, node_id, sf):
        p = self.params
        demanded = self.get_demanded_cap(flow.dr, node_id, sf)
        node = p.network.nodes[node_id]
        assert node["remaining_cap"] >= 0, "remaining node capacity below 0"
        if demanded <= node["cap"]:
            flow.processing_index += 1
            p.metrics.add_active_flow(flow, node_id, sf)
            node["available_sf"][sf]["load"] += flow.dr
            node["remaining_cap"] = node["cap"] - demanded
            p.metrics.calc_max_node_usage(node_id, demanded)
            start = node["available_sf"][sf]["startup_time"]
            startup = p.sf_list[sf]["startup_delay"]
            if not (start + startup <= self.env.now):
                remaining = (start + startup) - self.env.now
                if flow.ttl - remaining <= 0:
                    flow.ttl = 0
                    return False
                flow.end2end_delay += remaining
                flow.ttl -= remaining
                yield self.env.timeout(remaining)
            return True
        return False

    def finish_processing(self, flow, node_id, sf):
        p = self.params
        flow.current_position += 1
        if flow.current_position == len(p.sfc_list[flow.sfc]):
            flow.forward_to_eg = True
        yield self.env.timeout(flow.duration)
        p.metrics.remove_active_flow(flow, node_id, sf)
        node = p.network.nodes[node_id]
        node["available_sf"][sf]["load"] -= flow.dr
        assert node["available_sf"][sf]["load"] >= 0, "SF load below 0"
        if node["available_sf"][sf]["load"] == 0 and sf not in p.sf_placement[node_id]:
            del node["available_sf"][sf]
        used = 0.0
        for sf_i, data in node["available_sf"].items():
            if sf_i != "EG":
                used += p.sf_list[sf_i]["resource_function"](data["load"])
        node["remaining_cap"] = node["cap"] - used
        assert node["remaining_cap"] <= node["cap"]


@register_plugin
class DefaultFlowProcessor(BaseFlowProcessor):
    def process_flow(self, flow):
        p = self.params
        node_id = flow.current_node_id
        sf = p.sfc_list[flow.sfc][flow.current_position]
        flow.current_sf = sf
        if sf in p.sf_placement[node_id]:
            delay = self.get_processing_delay(flow, sf)
            if not delay:  # reference semantics: a zero processing delay also drops (process_flow:32)
                return False
            ok = yield self.env.process(self.request_resources(flow, node_id, sf))
            if ok:
                yield self.env.timeout(delay)
                self.env.process(self.finish_processing(flow, node_id, sf))
                return True
            return False
        return False
