"""Simulator parameters (reference: ``coordsim/simulation/simulatorparams.py``).

Holds the network, SFC/SF lists, traffic parameters, plugin class names, the
two-state MMPP arrival model and the per-episode pre-generated flow lists.
RNG consumption order (Python ``random`` for inter-arrivals, NumPy's global
legacy generator for rates/sizes/choices) follows the reference exactly so the
oracle reproduces reference trajectories for stochastic configs too.
"""
import random

import numpy as np

DEFAULT_PLUGINS = {
    "flow_generator_class": "DefaultFlowGenerator",
    "flow_forwarder_class": "DefaultFlowForwarder",
    "flow_processor_class": "DefaultFlowProcessor",
    "decision_maker_class": "DefaultDecisionMaker",
    "controller_class": "DurationController",
}


class SimulatorParams:
    def __init__(self, logger, network, ing_nodes, eg_nodes, sfc_list, sf_list, config, metrics,
                 prediction=False, schedule=None, sf_placement=None):
        self.logger = logger
        self.network = network
        self.ing_nodes = ing_nodes
        self.eg_nodes = eg_nodes
        self.sfc_list = sfc_list
        self.sf_list = sf_list
        self.config = config
        for key, default in DEFAULT_PLUGINS.items():
            setattr(self, key, config.get(key, default))
        self.ttl_choices = config.get("ttl_choices", None)
        assert self.ttl_choices is not None, "TTL must be set in config file"
        self.vnf_timeout = config.get("vnf_timeout", 100)
        self.flow_trigger = None
        self.run_times = None
        self.episode = None
        self.metrics = metrics
        self.use_trace = "trace_path" in config
        self.writer = None
        self.prediction = prediction
        self.predicted_inter_arr_mean = {n[0]: config["inter_arrival_mean"] for n in ing_nodes}
        self.schedule = schedule if schedule is not None else {}
        self.sf_placement = sf_placement if sf_placement is not None else {}
        for node_id, sfs in self.sf_placement.items():
            for sf in sfs:
                avail = self.network.nodes[node_id]["available_sf"]
                avail[sf] = avail.get(sf, {"load": 0.0, "startup_time": 0.0, "last_active": 0.0})

        self.flow_dr_mean = config["flow_dr_mean"]
        self.flow_dr_stdev = config["flow_dr_stdev"]
        self.flow_size_shape = config["flow_size_shape"]
        self.deterministic_arrival = config.get("deterministic", None)
        self.deterministic_size = config.get("deterministic", None)
        if "deterministic_arrival" in config:
            self.deterministic_arrival = config["deterministic_arrival"]
        if "deterministic_size" in config:
            self.deterministic_size = config["deterministic_size"]
        if self.deterministic_arrival is None or self.deterministic_size is None:
            raise ValueError("'deterministic_arrival' or 'deterministic_size' are not set in simulator config.")
        self.run_duration = config["run_duration"]

        self.use_states = bool(config.get("use_states", False))
        self.states = {}
        self.in_init_state = True
        if self.use_states:
            self.init_state = config["init_state"]
            self.states = config["states"]
            self.inter_arr_mean = {n[0]: 0 for n in ing_nodes}
            if config.get("rand_init_state", False):
                # reference quirk Q16 reads self.network.ing_nodes (AttributeError); we use the ingress list
                names = list(self.states.keys())
                self.current_states = {n[0]: np.random.choice(names) for n in ing_nodes}
            else:
                self.current_states = {n[0]: self.init_state for n in ing_nodes}
            self.update_inter_arr_mean()
        else:
            self.update_single_inter_arr_mean(config["inter_arrival_mean"])

        self.flow_arrival_list = None
        self.flow_size_list = None
        self.flow_dr_list = None
        self.flow_list_idx = None
        self.last_arrival_sum = None
        self.generated_flows = []

    def __str__(self):
        return (f"SimulatorParams(inter_arr_mean={self.inter_arr_mean}, det_arrival={self.deterministic_arrival}, "
                f"dr={self.flow_dr_mean}±{self.flow_dr_stdev}, size_shape={self.flow_size_shape}, "
                f"det_size={self.deterministic_size})")

    # MMPP ------------------------------------------------------------------------------------
    def start_mmpp(self, env):
        self.env = env
        yield env.timeout(self.run_duration)
        yield env.process(self.update_state())

    def update_state(self):
        names = list(self.states.keys())
        for node in self.ing_nodes:
            cur = self.current_states[node[0]]
            p = self.states[cur]["switch_p"]
            if np.random.choice([False, True], p=[1 - p, p]):
                cur = names[1] if cur == names[0] else names[0]
                self.current_states[node[0]] = cur
        self.update_inter_arr_mean()
        yield self.env.timeout(self.run_duration)
        yield self.env.process(self.update_state())

    def update_inter_arr_mean(self):
        for node_id, state in self.current_states.items():
            self.inter_arr_mean[node_id] = self.states[state]["inter_arr_mean"]

    def update_single_inter_arr_mean(self, new_mean):
        self.inter_arr_mean = {n[0]: new_mean for n in self.ing_nodes}

    def update_single_predicted_inter_arr_mean(self, new_mean):
        self.predicted_inter_arr_mean = {n[0]: new_mean for n in self.ing_nodes}

    # pre-generated flow lists (ListFlowGenerator / prediction) ----------------------------------
    def reset_flow_lists(self):
        ids = [n[0] for n in self.ing_nodes]
        self.flow_arrival_list = {i: [] for i in ids}
        self.flow_size_list = {i: [] for i in ids}
        self.flow_dr_list = {i: [] for i in ids}
        self.flow_list_idx = {i: 0 for i in ids}
        self.last_arrival_sum = {i: 0 for i in ids}

    def generate_flow_lists(self, now=0):
        for ing in [n[0] for n in self.ing_nodes]:
            arrivals, sizes, drs = [], [], []
            run_end = now + self.run_duration
            while self.last_arrival_sum[ing] < run_end:
                if self.deterministic_arrival:
                    inter_arr = self.inter_arr_mean[ing]
                else:
                    inter_arr = random.expovariate(1.0 / self.inter_arr_mean[ing])
                dr = np.random.normal(self.flow_dr_mean, self.flow_dr_stdev)
                size = self.flow_size_shape if self.deterministic_size else np.random.pareto(self.flow_size_shape) + 1
                if dr < 0.0 or size < 0.0:
                    continue
                arrivals.append(inter_arr)
                sizes.append(size)
                drs.append(dr)
                self.last_arrival_sum[ing] += inter_arr
            self.flow_arrival_list[ing].extend(arrivals)
            self.flow_dr_list[ing].extend(drs)
            self.flow_size_list[ing].extend(sizes)
            self.generated_flows = drs

    def get_next_flow_data(self, ing):
        if self.flow_list_idx is None:
            self.reset_flow_lists()
            self.generate_flow_lists()
        idx = self.flow_list_idx[ing]
        assert idx < len(self.flow_arrival_list[ing])
        self.flow_list_idx[ing] += 1
        return self.flow_arrival_list[ing][idx], self.flow_dr_list[ing][idx], self.flow_size_list[ing][idx]

    def update_passed_traffic(self, dr, src, dst):
        self.network[src][dst]["run_passed_traffic"] += dr
