"""Batched device simulator (native HIP kernel; host path for CPU tests)."""
from .batched import BatchedSimulator, SimStepOut, sim_config_from_files
