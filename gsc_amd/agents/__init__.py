"""Agents: DDPG learner, batched device trainer, reference-equivalent single-env agent."""
from .ddpg import BatchedTrainer, DDPGLearner, TrainerConfig
from .replay import Batch, DeviceReplay, GraphReplayBuffer
from .simple_ddpg import SimpleDDPG
