"""Controllers: how long the simulator runs between external decisions.

Reference: ``coordsim/controller/{base,duration,flow}_controller.py``.
``DurationController`` (default) applies a placement+schedule and runs for
``run_duration`` ms; ``FlowController`` runs until the next flow needs a
per-flow decision (used with ``ExternalDecisionMaker``).
"""
import logging

from gsc_amd.spinterface import SimulatorAction, SimulatorState

log = logging.getLogger(__name__)

CONTROLLERS = {}


def register_controller(cls):
    CONTROLLERS[cls.__name__] = cls
    return cls


class BaseController:
    def __init__(self, env, params, simulator):
        self.env = env
        self.params = params
        self.simulator = simulator

    def get_init_state(self):
        raise NotImplementedError

    def get_next_state(self, action=None):
        raise NotImplementedError

    def network_metrics(self):
        s = self.params.metrics.get_metrics()
        self.traffic = s["run_total_requested_traffic"]
        self.network_stats = {
            "processed_traffic": s["run_total_processed_traffic"],
            "total_flows": s["generated_flows"],
            "successful_flows": s["processed_flows"],
            "dropped_flows": s["dropped_flows"],
            "run_successful_flows": s["run_processed_flows"],
            "run_dropped_flows": s["run_dropped_flows"],
            "run_dropped_flows_per_node": s["run_dropped_flows_per_node"],
            "in_network_flows": s["total_active_flows"],
            "avg_end2end_delay": s["avg_end2end_delay"],
            "run_avg_end2end_delay": s["run_avg_end2end_delay"],
            "run_max_end2end_delay": s["run_max_end2end_delay"],
            "run_avg_path_delay": s["run_avg_path_delay"],
            "run_total_processed_traffic": s["run_total_processed_traffic"],
        }

    def parse_network(self):
        usage = self.params.metrics.get_metrics()["run_max_node_usage"]
        net = self.params.network
        self.network_dict = {
            "nodes": [{"id": v, "resource": d["cap"], "used_resources": usage[v]} for v, d in net.nodes(data=True)],
            "edges": [{"src": u, "dst": v, "delay": d["delay"], "data_rate": d["cap"], "used_data_rate": 0}
                      for u, v, d in net.edges(data=True)],
        }
        return self.network_dict

    def _state(self):
        return SimulatorState(self.network_dict, self.params.sf_placement, self.params.sfc_list,
                              self.params.sf_list, self.traffic, self.network_stats)


@register_controller
class DurationController(BaseController):
    def __init__(self, env, params, simulator):
        super().__init__(env, params, simulator)
        self.episode = 0
        self.duration = params.run_duration

    def _predict(self):
        if getattr(self.params, "prediction", False):
            if getattr(self, "predictor", None) is None:
                from .predictor import TrafficPredictor
                self.predictor = TrafficPredictor(self.params)
            self.predictor.predict_traffic(self.env.now)

    def get_init_state(self):
        self.env.step()
        self._predict()
        self.parse_network()
        self.network_metrics()
        return self._state()

    def get_next_state(self, action: SimulatorAction) -> SimulatorState:
        p = self.params
        p.writer.write_schedule_table(p, self.env.now, action)
        p.sf_placement = action.placement
        for node_id, placed in action.placement.items():
            avail = {sf: d for sf, d in p.network.nodes[node_id]["available_sf"].items() if d["load"] != 0}
            for sf in placed:
                if sf not in avail:
                    avail[sf] = {"load": 0.0, "last_active": self.env.now, "startup_time": self.env.now}
            p.network.nodes[node_id]["available_sf"] = avail
        p.schedule = action.scheduling
        self.env.run(until=self.duration * p.run_times)
        self._predict()
        self.parse_network()
        self.network_metrics()
        return self._state()


class SPRState:
    """State returned by :class:`FlowController` (one pending flow + network view)."""

    def __init__(self, flow, network, sfcs, network_stats):
        self.flow = flow
        self.network = network
        self.sfcs = sfcs
        self.network_stats = network_stats


class FlowAction:
    """Per-flow action for :class:`FlowController` (the reference uses duck typing: ``.flow``/``.destination_node_id``)."""

    def __init__(self, flow, destination_node_id):
        self.flow = flow
        self.destination_node_id = destination_node_id


@register_controller
class FlowController(BaseController):
    def __init__(self, env, params, simulator):
        super().__init__(env, params, simulator)
        self.episode = 0

    def get_init_state(self):
        flow = self.env.run(until=self.params.flow_trigger)
        self.parse_network()
        self.network_metrics()
        return SPRState(flow, self.params.network, self.params.sfc_list, self.network_stats)

    def get_next_state(self, action):
        flow = action.flow
        node = flow.current_node_id
        nodes = self.params.network.nodes
        if action.destination_node_id == node:
            avail = nodes[node]["available_sf"]
            if flow.current_sf not in avail and flow.current_sf != "EG":
                avail[flow.current_sf] = {"load": 0.0, "last_active": self.env.now, "startup_time": self.env.now}
        self.update_vnf_active_status()
        self.params.sf_placement = {v: list(d["available_sf"].keys()) for v, d in nodes(data=True)}
        self.env.process(self.simulator.handle_flow(flow, decision=action.destination_node_id))
        flow = self.env.run(until=self.params.flow_trigger)
        self.parse_network()
        self.network_metrics()
        return SPRState(flow, self.params.network, self.params.sfc_list, self.network_stats)

    def update_vnf_active_status(self):
        now = self.env.now
        for v, d in self.params.network.nodes(data=True):
            for sf, sfp in dict(d["available_sf"]).items():
                if sfp["load"] == 0.0:
                    if sfp["last_active"] < now - self.params.vnf_timeout:
                        del d["available_sf"][sf]
                else:
                    d["available_sf"][sf]["last_active"] = now
