"""Test-mode CSV writer and run-window clock (reference: ``coordsim/writer/writer.py``).

``write_network_state`` is a simulation process that fires every
``run_duration``: in test mode it appends one row per CSV; in every mode it
resets the per-run metrics, which defines the window the next observation and
reward are computed over.
"""
import csv
import os

import yaml

HEADERS = {
    "placements.csv": ["episode", "time", "node", "sf"],
    "node_metrics.csv": ["episode", "time", "node", "node_capacity", "used_resources", "ingress_traffic"],
    "metrics.csv": ["episode", "time", "total_flows", "successful_flows", "dropped_flows", "in_network_flows",
                    "avg_end2end_delay"],
    "run_flows.csv": ["episode", "time", "successful_flows", "dropped_flows", "total_flows"],
    "runtimes.csv": ["run", "runtime"],
    "drop_reasons.csv": ["episode", "time", "TTL", "DECISION", "LINK_CAP", "NODE_CAP"],
    "rl_state.csv": None,
}
SCHEDULE_HEADER = ["episode", "time", "origin_node", "sfc", "sf", "schedule_node", "schedule_prob"]
FLOW_ACTION_HEADER = ["episode", "time", "flow_id", "flow_rem_ttl", "flow_ttl", "curr_node_id", "dest_node",
                      "cur_node_rem_cap", "next_node_rem_cap", "link_cap", "link_rem_cap"]


class ResultWriter:
    def __init__(self, test_mode: bool, test_dir=None, write_schedule=False, write_flow_actions=False):
        self.test_mode = test_mode
        self.write_schedule = write_schedule
        self.write_per_flow_actions = write_flow_actions
        self.test_dir = test_dir
        self._streams = {}
        self._writers = {}
        self.action_number = 0
        if test_mode:
            os.makedirs(test_dir, exist_ok=True)
            files = dict(HEADERS)
            if write_schedule:
                files["scheduling.csv"] = SCHEDULE_HEADER
            if write_flow_actions:
                files["flow_actions.csv"] = FLOW_ACTION_HEADER
            for name, header in files.items():
                stream = open(os.path.join(test_dir, name), "a+", newline="")
                self._streams[name] = stream
                self._writers[name] = csv.writer(stream)
                if header is not None:
                    self._writers[name].writerow(header)

    def close(self):
        for s in self._streams.values():
            s.close()
        self._streams.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _w(self, name):
        return self._writers[name]

    def write_runtime(self, runtime):
        if self.test_mode:
            self.action_number += 1
            self._w("runtimes.csv").writerow([self.action_number, runtime])

    def write_flow_action(self, params, time, flow, current_node_id, destination_node_id):
        if not (self.test_mode and self.write_per_flow_actions):
            return
        nodes = params.network.nodes
        cur_rem = nodes[flow.current_node_id]["remaining_cap"]
        link_cap = rem_cap = -1
        if destination_node_id is None:
            dest, next_rem = "None", -1
        else:
            dest = destination_node_id
            next_rem = nodes[dest]["remaining_cap"]
            if dest == flow.current_node_id:
                link_cap = rem_cap = "inf"
            else:
                e = params.network.edges[(flow.current_node_id, dest)]
                link_cap, rem_cap = e["cap"], e["remaining_cap"]
        self._w("flow_actions.csv").writerow([params.episode, time, flow.flow_id, flow.ttl, flow.original_ttl,
                                              flow.current_node_id, dest, cur_rem, next_rem, link_cap, rem_cap])

    def write_schedule_table(self, params, time, action):
        if self.test_mode and self.write_schedule:
            rows = []
            for node, sfcs in action.scheduling.items():
                for sfc, sfs in sfcs.items():
                    for sf, sched in sfs.items():
                        for dst, prob in sched.items():
                            rows.append([params.episode, time, node, sfc, sf, dst, prob])
            self._w("scheduling.csv").writerows(rows)

    def begin_writing(self, env, params):
        self.env = env
        self.params = params
        yield env.process(self.write_network_state())

    def write_network_state(self):
        time = self.env.now
        p = self.params
        if self.test_mode:
            m = p.metrics.get_metrics()
            self._w("metrics.csv").writerow([p.episode, time, m["generated_flows"], m["processed_flows"],
                                             m["dropped_flows"], m["total_active_flows"], m["avg_end2end_delay"]])
            rows = []
            for node_id, d in p.network.nodes(data=True):
                ingress_traffic = 0
                for sfc, sfs in p.sfc_list.items():
                    ingress_traffic += m["run_act_total_requested_traffic"].get(node_id, {}).get(sfc, {}).get(sfs[0], 0)
                rows.append([p.episode, time, node_id, d["cap"], m["run_max_node_usage"][node_id], ingress_traffic])
            r = m["dropped_flow_reasons"]
            self._w("drop_reasons.csv").writerow([p.episode, time, r["TTL"], r["DECISION"], r["LINK_CAP"],
                                                  r["NODE_CAP"]])
            self._w("run_flows.csv").writerow([p.episode, time, m["run_processed_flows"], m["run_dropped_flows"],
                                               m["run_generated_flows"]])
            self._w("node_metrics.csv").writerows(rows)
            self._w("placements.csv").writerows(
                [[p.episode, time, v, sf] for v, d in p.network.nodes(data=True) for sf in d["available_sf"]])
        p.metrics.reset_run_metrics()
        yield self.env.timeout(p.run_duration)
        yield self.env.process(self.write_network_state())

    def write_dropped_flow_locs(self, locs):
        if self.test_mode:
            with open(os.path.join(self.test_dir, "dropped_flows.yaml"), "w") as f:
                yaml.safe_dump(locs, f, default_flow_style=False)

    def write_rl_state(self, rl_state):
        if self.test_mode:
            self._w("rl_state.csv").writerow(rl_state)
