"""Trace-driven traffic (reference: ``coordsim/trace_processor/trace_processor.py``).

Walks rows ``time[,node],inter_arrival_mean[,cap]``: waits until ``time - 1``
and then sets the node's (or every node's) inter-arrival mean; ``'None'``
switches a node off; an optional ``cap`` column changes the node capacity.
"""
import numpy as np


class TraceProcessor:
    def __init__(self, params, env, trace, simulator):
        self.params = params
        self.env = env
        self.trace = trace
        self.trace_index = 0
        self.simulator = simulator
        env.process(self.process_trace())

    def process_trace(self):
        row = self.trace[self.trace_index]
        wait = float(np.clip(float(row["time"]) - self.env.now - 1, 0, None))
        mean = row["inter_arrival_mean"]
        yield self.env.timeout(wait)
        if "node" in row:
            node_id = row["node"]
            if mean == "None":
                self.params.inter_arr_mean[node_id] = None
            else:
                self.params.inter_arr_mean[node_id] = float(mean)
                if "cap" in row:
                    self.params.network.nodes[node_id]["cap"] = float(row["cap"])
        else:
            self.params.update_single_inter_arr_mean(float(mean))
        if self.trace_index < len(self.trace) - 1:
            self.trace_index += 1
            self.env.process(self.process_trace())
