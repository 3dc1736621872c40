"""Agents: DDPG learner, batched device trainer, reference-equivalent single-env agent."""
from .ddpg import BatchedTrainer, DDPGLearner, TrainerConfig
from .replay import Batch, DeviceReplay, GraphReplayBuffer
from .base import RLSPAgent
from .simple_ddpg import SimpleDDPG
