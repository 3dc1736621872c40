"""List-based future-traffic prediction (reference traffic_predictor.py; disabled upstream)."""
import yaml

from gsc_amd.coordsim import Simulator
from gsc_amd.coordsim import dummy_data
from gsc_amd.spinterface import SimulatorAction
from tests.conftest import cfg_path

NET3 = cfg_path("networks", "triangle", "triangle-in1-cap10-delay10.graphml")
ABC = cfg_path("service_functions", "abc.yaml")


def _sim(tmp_path, predict):
    cfg = yaml.safe_load(open(cfg_path("config", "simulator", "rand-arrival10_det-size001_duration100.yaml")))
    cfg.update(future_traffic=predict, flow_generator_class="ListFlowGenerator")
    p = tmp_path / f"sim{int(predict)}.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return Simulator(NET3, ABC, str(p))


def test_prediction_equals_next_window_traffic(tmp_path):
    """With ListFlowGenerator the ingress rate predicted at the start of a window equals the data
    rate of the flows the simulator then generates at that ingress during the window."""
    sim = _sim(tmp_path, True)
    s = sim.init(7)
    nodes = [n["id"] for n in s.network["nodes"]]
    pl, sc = dummy_data.POLICIES["chain"]
    act = SimulatorAction(pl(nodes, s.sfcs), sc(nodes, s.sfcs))
    predicted = s.traffic["pop0"]["sfc_1"]["a"]
    total = 0.0
    for k in range(8):
        s = sim.apply(act)
        generated = sim.metrics.metrics["run_total_requested_traffic_node"]["pop0"]
        # window 0: the t=0 arrival precedes the writer's first run-metric reset (reference t=0
        # quirk), so the generated-traffic metric misses that one flow
        assert abs(predicted - generated - (1.0 if k == 0 else 0.0)) < 1e-9, k
        total += generated
        predicted = s.traffic["pop0"]["sfc_1"]["a"]
    assert total > 0


def test_prediction_off_by_default():
    sim = Simulator(NET3, ABC, cfg_path("config", "simulator", "sample_config.yaml"))
    assert sim.prediction is False
