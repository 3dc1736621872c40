"""Per-flow state machine driving the plugins (reference: ``coordsim/simulation/flowsimulator.py``)."""
import logging

from tqdm import tqdm

from .flow import Flow
from .plugins import (BaseDecisionMaker, BaseFlowForwarder, BaseFlowGenerator, BaseFlowProcessor,
                      get_plugin)

log = logging.getLogger(__name__)


class FlowSimulator:
    def __init__(self, env, params, quiet: bool = True):
        self.env = env
        self.params = params
        self.quiet = quiet
        self.total_flow_count = 0
        params.flow_trigger = env.event()
        self.FlowGenerator = get_plugin(params.flow_generator_class, BaseFlowGenerator)(env, params)
        self.DecisionMaker = get_plugin(params.decision_maker_class, BaseDecisionMaker)(env, params)
        self.FlowForwarder = get_plugin(params.flow_forwarder_class, BaseFlowForwarder)(env, params)
        self.FlowProcessor = get_plugin(params.flow_processor_class, BaseFlowProcessor)(env, params)

    def start(self):
        if not self.quiet:
            tqdm.write(f"Ingress nodes: {[n[0] for n in self.params.ing_nodes]}")
            if self.params.eg_nodes:
                tqdm.write(f"Egress nodes: {self.params.eg_nodes}")
        for node in self.params.ing_nodes:
            self.env.process(self.init_arrival(node[0]))

    def init_arrival(self, node_id):
        while self.params.inter_arr_mean[node_id] is not None:
            self.total_flow_count += 1
            inter_arr, flow = self.FlowGenerator.generate_flow(self.total_flow_count, node_id)
            self.env.process(self.handle_flow(flow))
            yield self.env.timeout(inter_arr)

    def handle_flow(self, flow: Flow, decision=False):
        metrics = self.params.metrics
        while not flow.departed:
            if decision is False:
                next_node = yield self.env.process(self.DecisionMaker.decide_next_node(flow))
                if next_node == "External":
                    return
            else:
                next_node = decision
                decision = False
                if flow.forward_to_eg and flow.current_node_id == next_node:
                    yield self.env.timeout(1)
                    flow.ttl -= 1
                    flow.end2end_delay += 1
            if next_node is None:
                metrics.dropped_flow(flow, "DECISION")
                return
            dtype = self.DecisionMaker.decision_type
            process = dtype != "PerFlow" or next_node == flow.current_node_id
            forwarded = yield self.env.process(self.FlowForwarder.forward_flow(flow, next_node))
            if not forwarded:
                metrics.dropped_flow(flow, "LINK_CAP")
                return
            if not flow.forward_to_eg and process:
                processed = yield self.env.process(self.FlowProcessor.process_flow(flow))
                if not processed:
                    metrics.dropped_flow(flow, "NODE_CAP")
                    return
        self.depart_flow(flow)

    def depart_flow(self, flow):
        self.params.metrics.completed_flow()
        self.params.metrics.add_end2end_delay(flow.end2end_delay)
