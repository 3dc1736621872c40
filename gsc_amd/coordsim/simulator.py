"""Scalar coord-sim backend implementing :class:`SimulatorInterface`.

Reference: ``siminterface/simulator.py``.  ``init(seed)`` builds a fresh event
environment, reseeds Python's and NumPy's global RNGs (reference behaviour,
``simulator.py:111-113``), starts the writer clock, arrival processes, optional
MMPP/trace processes and advances one event; ``apply(action)`` runs one
``run_duration`` window via the configured controller.

This is the exact-semantics oracle; the batched device simulator
(:mod:`gsc_amd.sim`) is differential-tested against it.

Deliberate deviations (documented quirks):
* Q14: a relative ``trace_path`` that does not exist under the CWD is also
  looked up next to the sim-config file and under ``configs/traces/``.
* Q15: the trace file is *not* copied next to the network file.
"""
from __future__ import annotations

import logging
import os
import random
import time

import numpy

from gsc_amd.spinterface import SimulatorInterface, SimulatorState
from . import reader
from .controllers import BaseController, CONTROLLERS
from .engine import Environment
from .flowsim import FlowSimulator
from .metrics import Metrics
from .params import SimulatorParams
from .trace import TraceProcessor
from .writer import ResultWriter

logger = logging.getLogger(__name__)

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def resolve_trace_path(trace_path: str, config_file: str = "") -> str:
    cands = [os.path.join(os.getcwd(), trace_path)]
    if config_file:
        cands.append(os.path.join(os.path.dirname(os.path.abspath(config_file)), trace_path))
    cands.append(os.path.join(_REPO_ROOT, "configs", "traces", os.path.basename(trace_path)))
    for c in cands:
        if os.path.exists(c):
            return c
    raise FileNotFoundError(f"trace file {trace_path} not found (tried {cands})")


class Simulator(SimulatorInterface):
    def __init__(self, network_file, service_functions_file, config_file, resource_functions_path="",
                 test_mode=False, test_dir=None):
        super().__init__(test_mode)
        self.network_file = network_file
        self.test_dir = test_dir
        self.sfc_list = reader.get_sfc(service_functions_file)
        self.sf_list = reader.get_sf(service_functions_file, resource_functions_path)
        self.config = reader.get_config(config_file)
        self.network, self.ing_nodes, self.eg_nodes = reader.network_builder(network_file, self.config)
        self.metrics = Metrics(self.network, self.sf_list)
        # reference forces prediction off (simulator.py:47); ``future_traffic: true`` enables the
        # list-based predictor (coordsim/predictor.py)
        self.prediction = bool(self.config.get("future_traffic", False))
        self.params = SimulatorParams(logger, self.network, self.ing_nodes, self.eg_nodes, self.sfc_list,
                                      self.sf_list, self.config, self.metrics, prediction=self.prediction)
        self.writer = ResultWriter(test_mode, test_dir, bool(self.config.get("write_schedule", False)),
                                   bool(self.config.get("write_flow_actions", False)))
        self.params.writer = self.writer
        self.episode = 0
        self.params.episode = 0
        self.last_apply_time = None
        self.trace = None
        if "trace_path" in self.config:
            self.trace = reader.get_trace(resolve_trace_path(self.config["trace_path"], config_file))
        self.env = None

    def init(self, seed) -> SimulatorState:
        self.episode += 1
        self.params.episode += 1
        reader.reset_cap(self.network)
        self.params.run_times = 1
        self.start_time = time.time()
        self.env = Environment()
        self.env.process(self.writer.begin_writing(self.env, self.params))
        self.params.metrics.reset_metrics()
        if self.params.use_states:
            self.params.in_init_state = False
            self.env.process(self.params.start_mmpp(self.env))
        self.duration = self.params.run_duration
        self.seed = seed
        random.seed(seed)
        numpy.random.seed(seed)
        self.params.reset_flow_lists()
        self.params.generate_flow_lists()
        self.simulator = FlowSimulator(self.env, self.params)
        if self.trace is not None:
            TraceProcessor(self.params, self.env, self.trace, self.simulator)
        self.simulator.start()
        try:
            ctrl_cls = CONTROLLERS[self.params.controller_class]
        except KeyError:
            raise ValueError(f"unknown controller {self.params.controller_class}") from None
        assert issubclass(ctrl_cls, BaseController)
        self.controller = ctrl_cls(self.env, self.params, self.simulator)
        self.params.metrics.running_time(self.start_time, time.time())
        state = self.controller.get_init_state()
        self.last_apply_time = time.time()
        return state

    def apply(self, actions) -> SimulatorState:
        self.writer.write_runtime(time.time() - self.last_apply_time)
        state = self.controller.get_next_state(actions)
        self.params.run_times += 1
        self.params.metrics.running_time(self.start_time, time.time())
        self.params.generate_flow_lists(now=self.env.now)
        self.last_apply_time = time.time()
        return state

    def get_active_ingress_nodes(self):
        return [ing[0] for ing in self.ing_nodes if self.params.inter_arr_mean[ing[0]] is not None]

    def close(self):
        self.writer.write_dropped_flow_locs(self.metrics.metrics["dropped_flows_locs"])
        self.writer.close()
