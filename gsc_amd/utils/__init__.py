"""Experiment plumbing, checkpointing and tracing (SURVEY.md sections 2.2, 5.1, 5.4, 5.5)."""
from .checkpoint import (load_actor, load_agent_helper, load_checkpoint, save_actor, save_agent_helper,
                         save_checkpoint)
from .experiment import (AgentHelper, ExperimentResult, MetricsLogger, ResultsWriter, get_config, load_schedule,
                         set_random_seed, setup, setup_files, setup_logging)
from .tracing import SPSCounter, phase_report, trace_range
