"""Future-traffic predictor (reference ``coordsim/traffic_predictor/traffic_predictor.py``).

With prediction on, the ingress entries of ``run_total_requested_traffic`` (the observation's
ingress-traffic feature) are replaced by the data rate of the flows that *will* arrive during the
next run window, read ahead from the pre-generated per-ingress flow lists (pair it with
``flow_generator_class: ListFlowGenerator`` so the prediction is exact).  Like the reference, all
predicted traffic is attributed to the first SFC's first SF.

The reference forces prediction off (``siminterface/simulator.py:47``) and its LSTM variant needs
keras; here the list-based predictor is enabled with ``future_traffic: true`` in the simulator
config (scalar backend).  The LSTM predictor is not provided (no keras; dead code upstream).
"""
from __future__ import annotations

from collections import defaultdict


def _d3():
    return defaultdict(lambda: defaultdict(float))


class TrafficPredictor:
    def __init__(self, params):
        self.params = params
        self.flow_idx = {ing[0]: 0 for ing in params.ing_nodes}
        self.arrival_sum = {ing[0]: 0.0 for ing in params.ing_nodes}

    def predict_traffic(self, now: float) -> None:
        p = self.params
        run_end = now + p.run_duration
        req = defaultdict(_d3)
        sfc = next(iter(p.sfc_list))
        first_sf = p.sfc_list[sfc][0]
        for ing in p.ing_nodes:
            node = ing[0]
            dr = 0.0
            if p.inter_arr_mean.get(node) is not None:
                while self.arrival_sum[node] < run_end:
                    if self.flow_idx[node] >= len(p.flow_arrival_list[node]):
                        p.generate_flow_lists(now=run_end)  # read further ahead
                        if self.flow_idx[node] >= len(p.flow_arrival_list[node]):
                            break
                    dr += p.flow_dr_list[node][self.flow_idx[node]]
                    self.arrival_sum[node] += p.flow_arrival_list[node][self.flow_idx[node]]
                    self.flow_idx[node] += 1
            req[node][sfc][first_sf] = dr
        p.metrics.metrics["run_total_requested_traffic"] = req
