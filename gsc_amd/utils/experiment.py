"""Experiment plumbing: agent config, result-directory layout, logging, seeds, metadata.

Reference: ``src/rlsp/agents/main.py`` (setup / get_config / setup_files / copy_input_files /
set_random_seed / setup_logging), ``agent_helper.py``, ``experiment_result.py``,
``result_writer.py``, ``common/common_functionalities.py`` (create_input_file / num_ingress).

Result directory (kept compatible):
``results/<agent_cfg>/<scheduler>/<service>/<simcfg>/<YYYY-mm-dd_HH-MM-SS>_seed<seed>/`` with
``input.yaml``, ``training.log``, copies of every input file (schedule paths rewritten to the
copies), ``rewards.csv`` (header-less column ``r``), ``trained_actor.pt``, ``agent_helper.obj``
(JSON metadata here — no pickles), test-mode simulator CSVs, plus ``metrics.jsonl`` and
``checkpoint.pt`` (full training state; new).
"""
from __future__ import annotations

import csv
import json
import logging
import logging.config
import os
import random
import shutil
import time
from datetime import datetime
from typing import Dict, Optional

import numpy as np
import yaml

from gsc_amd.coordsim.reader import num_ingress
from gsc_amd.envs.rewards import SUPPORTED_OBJECTIVES

DATETIME = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
logger = logging.getLogger("gsc_amd")


def get_config(config_file: str) -> dict:
    """Agent YAML with the reference defaults and objective validation (main.py:249-276)."""
    with open(config_file) as f:
        config = yaml.safe_load(f)
    config.setdefault("shuffle_nodes", False)
    config.setdefault("observation_space", ["ingress_traffic"])
    obj = config.get("objective")
    assert obj in SUPPORTED_OBJECTIVES, f"Objective {obj} not recognized. Must be one of {SUPPORTED_OBJECTIVES}."
    if obj == "prio-flow":
        ts = config.get("target_success")
        assert ts == "auto" or (ts is not None and 0 <= ts <= 1)
    if obj in {"soft-deadline", "soft-deadline-exp"}:
        assert "soft_deadline" in config
        if obj == "soft-deadline-exp":
            assert config.get("dropoff", 0) > 0, "Use 'soft-deadline' objective for 0 dropoff."
    if obj == "weighted":
        for w in ("flow_weight", "delay_weight", "node_weight", "instance_weight"):
            if w not in config:
                logger.warning(f"Using weighted objective, but {w} not configured. Defaulting to {w}=0.")
    config.setdefault("target_success", None)
    config.setdefault("soft_deadline", None)
    config.setdefault("dropoff", None)
    for w in ("flow_weight", "delay_weight", "node_weight", "instance_weight"):
        config.setdefault(w, 0)
    return config


def load_schedule(path: str) -> dict:
    with open(path) as f:
        sched = yaml.safe_load(f)
    for k in ("training_network_files", "inference_network", "period"):
        if k not in sched:
            raise ValueError(f"scheduler config {path} misses '{k}'")
    return sched


def get_base_path(agent_config_path, schedule_path, service_path, sim_config_path) -> str:
    stem = lambda p: os.path.splitext(os.path.basename(p))[0]
    return f"{stem(agent_config_path)}/{stem(schedule_path)}/{stem(service_path)}/{stem(sim_config_path)}"


class ExperimentResult:
    """Run metadata written to ``result.yaml`` (instance attributes; reference Q20 made them class-level)."""

    def __init__(self, _id: str):
        self.id = _id
        self.env_config: Dict = {}
        self.agent_config: Dict = {}
        self.episodes = 0
        self.runtime_process = self.runtime_walltime = 0.0
        self.log_file = None
        self._p0 = self._w0 = None

    def runtime_start(self):
        self._p0, self._w0 = time.process_time(), time.perf_counter()

    def runtime_stop(self):
        self.runtime_process = time.process_time() - self._p0
        self.runtime_walltime = time.perf_counter() - self._w0

    def write_to_file(self, filename: str):
        data = {"id": self.id, "env_config": self.env_config, "agent_config": self.agent_config,
                "episodes": self.episodes, "runtime_process": self.runtime_process,
                "runtime_walltime": self.runtime_walltime, "log_file": self.log_file}
        with open(filename, "w") as f:
            yaml.safe_dump(data, f, default_flow_style=False)


class AgentHelper:
    """Mutable bag threaded through setup/training (reference ``agent_helper.py``)."""

    def __init__(self, agent_config, network, service, sim_config, schedule, seed, episodes, weights=None,
                 verbose=False, DATETIME=DATETIME, test=None, append_test=False, sim_seed=None, gen_scenario=None,
                 episode_steps=200):
        self.episode_steps = episode_steps
        self.verbose = verbose
        self.agent_config_path = agent_config
        self.network_path = network
        self.service_path = service
        self.sim_config_path = sim_config
        self.schedule_path = schedule
        self.schedule = None
        self.seed = seed
        self.datetime = DATETIME
        self.experiment_id = f"{DATETIME}_seed{seed}"
        self.result = ExperimentResult(self.experiment_id)
        self.weights = weights
        self.episodes = episodes
        self.config = None
        self.config_dir = None
        self.result_base_path = None
        self.graph_base_path = None
        self.result_file = None
        self.logfile = None
        self.weights_path = None
        self.graph_path = None
        self.env = None
        self.test = test
        self.train = not bool(test)
        self.test_mode = bool(test) and not append_test
        self.append_test = append_test
        if append_test:
            self.test = self.experiment_id
        self.gen_scenario = gen_scenario
        self.gen_scenario_test = False
        self.sim_seed = sim_seed

    def to_json(self) -> dict:
        keep = ("episode_steps", "agent_config_path", "network_path", "service_path", "sim_config_path",
                "schedule_path", "schedule", "seed", "experiment_id", "episodes", "config", "config_dir", "test",
                "sim_seed", "weights")
        return {k: getattr(self, k) for k in keep}

    @classmethod
    def from_json(cls, d: dict) -> "AgentHelper":
        h = cls(d["agent_config_path"], d["network_path"], d["service_path"], d["sim_config_path"],
                d["schedule_path"], d["seed"], d["episodes"], episode_steps=d["episode_steps"])
        for k, v in d.items():
            setattr(h, k, v)
        h.test_mode = True
        return h


def setup_logging(verbose: bool, logfile: Optional[str]) -> logging.Logger:
    conf = os.path.join(_REPO_ROOT, "logging.conf")
    if os.path.exists(conf):
        logging.config.fileConfig(conf, disable_existing_loggers=False)
    root = logging.getLogger()
    if verbose and root.handlers:
        root.handlers[0].setLevel(logging.DEBUG)
    if logfile:
        os.makedirs(os.path.dirname(os.path.realpath(logfile)), exist_ok=True)
        fh = logging.FileHandler(logfile, mode="a")
        fh.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
        fh.setLevel(logging.DEBUG if verbose else logging.INFO)
        root.addHandler(fh)
    return root


def set_random_seed(seed: int) -> None:
    """Seed Python, NumPy and torch (reference also hides GPUs; this framework uses them)."""
    import torch
    os.environ["PYTHONHASHSEED"] = str(seed)
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)


def copy_input_files(target_dir, agent_config_path, network_path, service_path, sim_config_path, scheduler_path,
                     schedule: dict):
    os.makedirs(target_dir, exist_ok=True)
    new = lambda p: os.path.join(target_dir, os.path.basename(p))
    files = []
    for item in schedule["training_network_files"]:
        shutil.copyfile(item, new(item))
        files.append(new(item))
    schedule["training_network_files"] = files
    shutil.copyfile(schedule["inference_network"], new(schedule["inference_network"]))
    schedule["inference_network"] = new(schedule["inference_network"])
    for p in (agent_config_path, service_path, sim_config_path, scheduler_path):
        shutil.copyfile(p, new(p))
    return new(agent_config_path), new(network_path), new(service_path), new(sim_config_path), new(scheduler_path)


def create_input_file(target_dir, num_ingress_nodes, algo):
    os.makedirs(target_dir, exist_ok=True)
    with open(os.path.join(target_dir, "input.yaml"), "w") as f:
        yaml.safe_dump({"num_ingress": num_ingress_nodes, "algorithm": algo}, f, default_flow_style=False)


def write_yaml(path: str, data: dict) -> None:
    os.makedirs(os.path.dirname(os.path.realpath(path)), exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump({k: (v.item() if hasattr(v, "item") else v) for k, v in data.items()}, f,
                       default_flow_style=False)


def setup_files(h: AgentHelper, results_root: str = "results", write_files: bool = True) -> None:
    base = get_base_path(h.agent_config_path, h.schedule_path, h.service_path, h.sim_config_path)
    h.result_base_path = os.path.join(results_root, base)
    h.graph_base_path = os.path.join("graph", base)
    h.config_dir = os.path.join(h.result_base_path, h.experiment_id) + os.sep
    h.logfile = os.path.join(h.config_dir, "training.log")
    h.graph_path = os.path.join(h.graph_base_path, h.experiment_id)
    if h.test and not h.append_test:
        h.config_dir = os.path.join(h.result_base_path, h.test, f"test-{h.datetime}_seed{h.seed}") + os.sep
        h.logfile = os.path.join(h.config_dir, "test.log")
        h.weights_path = os.path.join(h.result_base_path, h.test)
    h.result.log_file = h.logfile
    h.result_file = os.path.join(h.config_dir, "result.yaml")
    if not write_files:  # non-zero ranks: same paths, no files
        setup_logging(h.verbose, None)
        return
    setup_logging(h.verbose, h.logfile)
    (h.agent_config_path, h.network_path, h.service_path, h.sim_config_path,
     h.schedule_path) = copy_input_files(h.config_dir, h.agent_config_path, h.network_path, h.service_path,
                                         h.sim_config_path, h.schedule_path, h.schedule)


def setup(agent_config, network, service, sim_config, scheduler, seed, episodes, weights=None, verbose=False,
          test=None, append_test=False, sim_seed=None, gen_scenario=None, results_root="results",
          datetime_str: Optional[str] = None, write_files: bool = True) -> AgentHelper:
    """Reference ``setup`` (main.py:62-86).  ``datetime_str`` pins the run id (all DP ranks share one)."""
    h = AgentHelper(agent_config, network, service, sim_config, scheduler, seed, episodes, weights, verbose,
                    datetime_str or DATETIME, test, append_test, sim_seed, gen_scenario)
    h.schedule = load_schedule(scheduler)
    setup_files(h, results_root, write_files)
    set_random_seed(seed)
    h.config = get_config(h.agent_config_path)
    h.episode_steps = h.config["episode_steps"]
    h.result.episodes = episodes
    if write_files:
        create_input_file(h.config_dir, num_ingress(network), h.config.get("agent_type"))
    return h


class ResultsWriter:
    """Header-less CSV of episodic returns, column ``r`` (reference ``result_writer.py``)."""

    def __init__(self, filename: str, override_existing: bool = True):
        filename = os.path.realpath(filename)
        os.makedirs(os.path.dirname(filename), exist_ok=True)
        self.fh = open(filename, "w" if override_existing else "a", newline="\n")
        self.writer = csv.DictWriter(self.fh, fieldnames=("r",))

    def write_row(self, epinfo: dict) -> None:
        self.writer.writerow({"r": epinfo["r"]})
        self.fh.flush()

    def close(self) -> None:
        self.fh.close()


class MetricsLogger:
    """Scalar metrics as JSON lines (tensorboard is not a dependency); mirrors the reference tags."""

    def __init__(self, path: Optional[str]):
        self.fh = None
        if path:
            os.makedirs(os.path.dirname(os.path.realpath(path)), exist_ok=True)
            self.fh = open(path, "a")

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self.log({tag: value}, step)

    def log(self, scalars: dict, step: int) -> None:
        if self.fh:
            self.fh.write(json.dumps({"step": int(step), "time": time.time(), **{k: float(v) for k, v in scalars.items()}}) + "\n")
            self.fh.flush()

    def close(self):
        if self.fh:
            self.fh.close()
