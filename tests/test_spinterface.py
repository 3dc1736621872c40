"""SimulatorInterface contract (reference ``src/tests/test_simulatorInterface.py``) against the fake
backend and the real scalar backend, plus the stand-alone coord-sim CLI and its fixed policies."""
import pytest

from gsc_amd.coordsim import DummySimulator, Simulator
from gsc_amd.coordsim import dummy_data
from gsc_amd.spinterface import SimulatorAction, SimulatorInterface, SimulatorState
from tests.conftest import cfg_path

STATS_KEYS = ("total_flows", "successful_flows", "dropped_flows", "in_network_flows", "avg_end2end_delay")
NET3 = cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml")
ABC = cfg_path("service_functions", "abc.yaml")
SIMCFG = cfg_path("config", "simulator", "sample_config.yaml")


def _action(nodes, sfcs):
    pl, sc = dummy_data.POLICIES["chain"]
    return SimulatorAction(pl(nodes, sfcs), sc(nodes, sfcs))


def _check_state(state, n_nodes, n_edges):
    assert isinstance(state, SimulatorState)
    assert len(state.network["nodes"]) == n_nodes and len(state.network["edges"]) == n_edges
    for node in state.network["nodes"]:
        assert {"id", "resource", "used_resources"} <= set(node)
    for e in state.network["edges"]:
        assert {"src", "dst", "delay", "data_rate", "used_data_rate"} <= set(e)
    assert state.sfcs == {"sfc_1": ["a", "b", "c"]}
    assert set(state.service_functions) == {"a", "b", "c"}
    for k in STATS_KEYS:
        assert k in state.network_stats
    assert isinstance(state.traffic, dict) and isinstance(state.placement, dict)


@pytest.mark.parametrize("backend", ["dummy", "coordsim"])
def test_contract(backend):
    sim = DummySimulator("", "", "") if backend == "dummy" else Simulator(NET3, ABC, SIMCFG)
    assert isinstance(sim, SimulatorInterface)
    s0 = sim.init(1234)
    _check_state(s0, 3, 3)
    nodes = [n["id"] for n in s0.network["nodes"]]
    s1 = sim.apply(_action(nodes, s0.sfcs))
    _check_state(s1, 3, 3)
    assert sim.get_active_ingress_nodes() == ["pop0"]


def test_coordsim_apply_runs_one_window():
    sim = Simulator(NET3, ABC, SIMCFG)
    s = sim.init(1)
    nodes = [n["id"] for n in s.network["nodes"]]
    tot = 0
    for i in range(5):
        s = sim.apply(_action(nodes, s.sfcs))
        assert sim.env.now == pytest.approx(100.0 * (i + 1))
        tot += s.network_stats["run_successful_flows"]
    assert tot > 0 and s.network_stats["dropped_flows"] == 0


def test_dummy_policies_shapes():
    nodes = ["pop0", "pop1", "pop2", "pop3"]
    sfcs = {"s1": ["a", "b", "c"], "s2": ["a", "c"]}
    for name, (pl, sc) in dummy_data.POLICIES.items():
        sched = sc(nodes, sfcs)
        for src in nodes:
            for c, chain in sfcs.items():
                for sf in chain:
                    assert sum(sched[src][c][sf].values()) == pytest.approx(1.0), name
        assert set(pl(nodes, sfcs)) == set(nodes)
    assert dummy_data.chain_placement(nodes[:3], {"sfc_1": ["a", "b", "c"]}) == \
        {"pop0": ["a"], "pop1": ["b"], "pop2": ["c"]}


def test_standalone_cli_triangle_golden():
    """Triangle + abc + sample_config with the SF-per-node chain: every flow succeeds (SURVEY §4 golden 1.0)."""
    from gsc_amd.coordsim.main import main
    m = main(["-d", "20000", "-sf", ABC, "-n", NET3, "-c", SIMCFG, "-s", "1", "--json"])
    assert m["generated_flows"] == 2000
    assert m["dropped_flows"] == 0 and m["processed_flows"] >= 1990
