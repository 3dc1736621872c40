"""Fake simulator backend for tests (reference: ``dummy_env/dummy_simulator.py``).

Returns a fixed 3-node state from both ``init`` and ``apply``; the
``SimulatorInterface`` contract test runs against it.
"""
from gsc_amd.spinterface import SimulatorAction, SimulatorInterface, SimulatorState


class DummySimulator(SimulatorInterface):
    def __init__(self, network_file: str = "", service_functions_file: str = "", config_file: str = "",
                 test_mode=False):
        super().__init__(test_mode)
        self.network_file = network_file

    def init(self, seed: int, trace=None) -> SimulatorState:
        return self.example_state_1

    def apply(self, actions: SimulatorAction) -> SimulatorState:
        return self.example_state_1

    def get_active_ingress_nodes(self):
        return ["pop0"]

    @property
    def example_state_1(self) -> SimulatorState:
        nodes = [{"id": f"pop{i}", "resource": 42.0, "used_resources": 0.21} for i in range(3)]
        edges = [{"src": f"pop{a}", "dst": f"pop{b}", "delay": 13, "data_rate": 100, "used_data_rate": 62}
                 for a, b in ((0, 1), (1, 2), (2, 0))]
        return SimulatorState(
            network={"nodes": nodes, "edges": edges},
            sfcs={"sfc_1": ["a", "b", "c"]},
            service_functions={"a": {"processing_delay": 0.5}, "b": {"processing_delay": 0.3},
                               "c": {"processing_delay": 0.2}},
            traffic={"pop0": {"sfc_1": {"a": 1, "b": 1}}, "pop1": {"sfc_1": {"b": 1, "c": 1}},
                     "pop2": {"sfc_1": {"c": 1}}},
            network_stats={"total_flows": 136, "successful_flows": 30, "dropped_flows": 3, "in_network_flows": 32,
                           "avg_end2end_delay": 21, "run_avg_end2end_delay": 42,
                           "run_total_processed_traffic": {}, "run_avg_path_delay": 22, "processed_traffic": {}},
            placement={"pop0": ["a"], "pop1": ["b"], "pop2": ["c"]},
        )
