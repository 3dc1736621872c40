"""gsc_amd: MI355X-native GNN + DDPG service-coordination engine (capabilities of farzad1132/GSC).

Layers (bottom-up):
  coordsim/  scalar discrete-event oracle (coord-sim semantics) + readers
  sim/       batched HIP simulator (thousands of envs per GPU, lockstep)
  envs/      gym-style env, simulator wrapper, rewards, batched env
  ops/       hand-written HIP/CDNA4 kernels (GATv2, fused MLP, Adam, explore/post-process, replay)
  models/    GNN embedder, actor, critic
  agents/    DDPG (reference-equivalent single env + batched device trainer)
  parallel/  data parallelism over RCCL/xGMI
  utils/     config, results layout, logging, checkpointing, tracing
"""
__version__ = "0.1.0"
