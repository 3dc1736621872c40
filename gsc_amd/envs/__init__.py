"""RL environment layer: spaces, limits, codec, rewards, gym env."""
from .common import ActionScheduleProcessor, normalize_scheduling_probabilities, threshold_normalize
from .graph import GraphBatch, GraphObs
from .gym_env import GymEnv, make_simulator
from .limits import EnvironmentLimits
from .rewards import RewardCalculator, SUPPORTED_OBJECTIVES
from .wrapper import SimulatorWrapper
