"""``SimpleDDPG`` — the reference agent API over two environment backends.

Reference: ``src/rlsp/agents/simple_ddpg.py`` (construction ``:102-152``, ``_choose_action``
``:182-201``, ``train`` ``:280-329``, updates ``:204-234``, ``post_process_actions`` ``:374-395``,
``predict`` ``:331-336``) and ``AutoResetWithSeed`` (``:51-74``).

``backend="oracle"`` reproduces the reference loop on one :class:`~gsc_amd.envs.GymEnv` over the
scalar coord-sim: uniform-random warm-up actions for ``nb_steps_warmup_critic`` steps, then
``unscale(scale(mu(s)) + N(rand_mu, rand_sigma))`` clipped to ``[0, 1]``; two-pass threshold
(0.1) + normalise post-processing; the same seed at every reset; and at every episode end (past
warm-up) ``episode_steps`` DDPG updates on batches of 100 from a host ring buffer.  The learner
(fused GNN kernels, bf16 GEMMs, fused Adam+Polyak) runs on the GPU when there is one.

``backend="batched"`` is the MI355X path: ``num_envs`` lockstep environments of the device
simulator per GPU (:class:`~gsc_amd.agents.ddpg.BatchedTrainer`), 100 replayed samples per env
step, one process per GPU with RCCL gradient all-reduce.  ``episodes`` counts episodes *per env*
(``episodes * episode_steps`` lockstep iterations).

Both write ``rewards.csv`` (header-less ``r`` column, one row per finished episode; the batched
backend writes the mean return of the episodes finishing together), ``metrics.jsonl`` (the
reference's tensorboard tags + success ratio / SPS), and — new — periodic ``checkpoint.pt``.
Greedy :meth:`predict` applies no noise and no post-processing, like the reference.
"""
from __future__ import annotations

import logging
import os
import time
from typing import List, Optional

import numpy as np
import torch
from tqdm import tqdm

from gsc_amd.coordsim import reader
from gsc_amd.envs.common import schedule_threshold, threshold_normalize
from gsc_amd.envs.graph import GraphObs
from gsc_amd.models import GraphSet
from gsc_amd.parallel.dist import DistInfo
from gsc_amd.utils import checkpoint as ckpt
from gsc_amd.utils.experiment import MetricsLogger, ResultsWriter
from gsc_amd.utils.tracing import SPSCounter, trace_range
from .base import RLSPAgent
from .ddpg import BatchedTrainer, DDPGLearner, TrainerConfig
from .replay import GraphReplayBuffer

logger = logging.getLogger(__name__)

REFERENCE_BATCH = 100          # simple_ddpg.py:135 (hard-coded)
SCHEDULE_THRESHOLD = 0.1       # simple_ddpg.py:130


def default_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class SimpleDDPG(RLSPAgent):
    def __init__(self, agent_helper, backend: str = "auto", num_envs: Optional[int] = None, device=None,
                 dist_info: Optional[DistInfo] = None, checkpoint_every: int = 0, results_writers: bool = True,
                 trainer_overrides: Optional[dict] = None):
        h = self.agent_helper = agent_helper
        self.cfg = h.config
        self.dist = dist_info or DistInfo()
        self.device = torch.device(device) if device is not None else default_device()
        if backend == "auto":
            backend = "batched" if self.device.type == "cuda" else "oracle"
        if backend not in ("oracle", "batched"):
            raise ValueError(f"unknown backend {backend!r} (oracle|batched)")
        self.backend = backend
        self.episode_steps = int(self.cfg["episode_steps"])
        self.checkpoint_every = int(checkpoint_every)
        self.checkpoint_replay = "auto"          # auto | yes | no
        self.checkpoint_replay_max = 1 << 30     # bytes (auto)
        sched = h.schedule
        self.train_files: List[str] = list(sched["training_network_files"])
        self.period = int(sched.get("period", 0) or 0)
        files = self.train_files + [f for f in [sched["inference_network"]] if f not in self.train_files]
        self.network_files = files
        self.topo_index = {f: i for i, f in enumerate(files)}
        self.sim_cfg = reader.get_config(h.sim_config_path)
        self.sfc_list = reader.get_sfc(h.service_path)
        self.sf_list = reader.get_sf(h.service_path)
        self.n_pad = int(self.cfg.get("max_nodes", 24))
        self.C = len(self.sfc_list)
        self.F = max(len(v) for v in self.sfc_list.values())
        self.n_obs = len(self.cfg["observation_space"])
        self.action_dim = self.n_pad * self.C * self.F * self.n_pad
        self.global_step = 0
        self.episode = 0
        self.best_return = -np.inf
        self.sps = SPSCounter()
        main = self.dist.is_main and results_writers and h.config_dir
        self.rewards_writer = ResultsWriter(os.path.join(h.config_dir, "rewards.csv")) if main else None
        self.metrics = MetricsLogger(os.path.join(h.config_dir, "metrics.jsonl") if main else None)
        seed = int(h.seed)
        overrides = dict(trainer_overrides or {})
        if backend == "batched":
            from gsc_amd.sim.batched import load_batched_from_paths
            self.num_envs = int(num_envs or 256)
            self.sim = load_batched_from_paths(files, h.service_path, h.sim_config_path, self.cfg, self.num_envs,
                                               device=self.device, seed=seed * 1000 + self.dist.rank,
                                               same_seed_every_episode=overrides.pop("same_seed_every_episode",
                                                                                     False))
            overrides.setdefault("lazy_handoff", True)   # joins at metrics / checkpoints / after training
            tcfg = TrainerConfig(num_envs=self.num_envs, seed=seed + 17 * self.dist.rank, **overrides)
            self.trainer = BatchedTrainer(self.cfg, self.sim, tcfg, self.dist,
                                          network_schedule=list(range(len(self.train_files))), period=self.period)
            self.learner = self.trainer.learner
            self.graphs = self.trainer.graphs
        else:
            self.num_envs = 1
            topos = [reader.load_topology(f, self.sim_cfg) for f in files]
            self.graphs = GraphSet(topos, self.n_pad, self.device)
            self.learner = DDPGLearner(self.cfg, self.n_obs, self.action_dim, self.graphs, self.C, self.F,
                                       self.device, self.dist, seed=seed)
            self.rb = GraphReplayBuffer(int(self.cfg.get("mem_limit", 10000)), self.action_dim, self.n_pad,
                                        self.n_obs, rng=np.random.RandomState(seed))
            self.np_rng = np.random.default_rng(seed)
            self.batch_size = int(overrides.get("batch_size") or REFERENCE_BATCH)
            self.warmup = int(self.cfg.get("nb_steps_warmup_critic", 200))
            self.rand_mu = float(self.cfg.get("rand_mu", 0.0))
            self.rand_sigma = float(self.cfg.get("rand_sigma", 0.3))
            self.env = None
        self.actor = self.learner.actor

    # ------------------------------------------------------------------------------------------
    # acting
    def _node_rows(self, obs) -> torch.Tensor:
        """[n, n_obs] node features of a GraphObs, or of the flat (feature-major) observation the
        environment returns in flat mode (``graph_mode: False``)."""
        if isinstance(obs, GraphObs):
            return obs.x
        flat = torch.as_tensor(np.asarray(obs), dtype=torch.float32)
        return flat.view(self.n_obs, -1).t()

    def _obs_tensor(self, obs):
        rows = self._node_rows(obs)
        x = torch.zeros(1, self.n_pad, self.n_obs, dtype=torch.float32)
        x[0, :rows.shape[0]] = rows
        return x.to(self.device)

    @torch.no_grad()
    def predict(self, obs, topo: Optional[int] = None) -> np.ndarray:
        """Greedy action (no noise, no post-processing; ``simple_ddpg.py:331-336``).

        ``obs``: a :class:`GraphObs` (one env; ``topo`` = index into :attr:`network_files`,
        default: the inference network) or a padded ``[E, n_pad, F]`` tensor with ``topo [E]``."""
        if isinstance(obs, GraphObs) or (isinstance(obs, np.ndarray) and obs.ndim == 1):
            t = self.topo_index[self.agent_helper.schedule["inference_network"]] if topo is None else int(topo)
            out = self.learner.act(self._obs_tensor(obs), torch.tensor([t], device=self.device))
            return out[0].cpu().numpy()
        topo_t = torch.as_tensor(topo, device=self.device).view(-1).to(torch.int64)
        return self.learner.act(obs.to(self.device), topo_t).cpu().numpy()

    def _choose_action(self, obs: GraphObs, topo: int) -> np.ndarray:
        mask = self.graphs.action_masks(self.C, self.F)[topo].cpu().numpy()
        if self.global_step < self.warmup:
            return self.np_rng.random(self.action_dim, dtype=np.float32) * mask
        mu = self.predict(obs, topo)
        scaled = self.actor.scale_action(mu)
        scaled = scaled + self.np_rng.normal(self.rand_mu, self.rand_sigma, size=self.action_dim)
        # reference clips to [-1, 1] here and discards the result (simple_ddpg.py:197)
        return np.clip(self.actor.unscale_action(scaled), 0.0, 1.0)

    def post_process_actions(self, action: np.ndarray) -> np.ndarray:
        return threshold_normalize(action, self.n_pad, schedule_threshold(self.cfg, self.n_pad), passes=2)

    # ------------------------------------------------------------------------------------------
    # training
    def train(self, episodes: int) -> dict:
        self.sps = SPSCounter()
        if self.backend == "batched":
            return self._train_batched(int(episodes))
        return self._train_oracle(int(episodes))

    def _episode_end(self, ep_return: float, info: dict) -> None:
        if self.rewards_writer is not None:
            self.rewards_writer.write_row({"r": ep_return})
        new_best = ep_return > self.best_return
        self.best_return = max(self.best_return, ep_return)
        sps = self.sps.rate(reset=True)
        scalars = {"charts/episodic_return": ep_return, "charts/episodic_length": self.episode_steps,
                   "charts/SPS": sps, **info}
        self.metrics.log(scalars, self.global_step)
        if self.dist.is_main:
            tqdm.write(f"episode {self.episode}: return {ep_return:.3f}" + (" (NEW best reward)" if new_best else "")
                       + f"  success {info.get('charts/success_ratio', float('nan')):.3f}  {sps:.1f} env-steps/s")
        if self.checkpoint_every and self.episode % self.checkpoint_every == 0 and self.agent_helper.config_dir:
            self.save_checkpoint(os.path.join(self.agent_helper.config_dir, "checkpoint.pt"))

    def _make_env(self, test_mode: bool = False):
        from gsc_amd.envs import GymEnv
        h = self.agent_helper
        return GymEnv(self.cfg, h.schedule, h.network_path, h.service_path, seed=h.seed, sim_seed=h.sim_seed,
                      agent_helper=h, sim_config_file=h.sim_config_path, test_mode=test_mode)

    def _train_oracle(self, episodes: int) -> dict:
        h = self.agent_helper
        if self.env is None:
            self.env = self._make_env(test_mode=False)
            self.env.episode_count = self.episode  # network scheduler position (resume)
            self.obs, _ = self.env.reset(seed=h.seed)
        total = episodes * self.episode_steps
        ep_ret, succ, drop = 0.0, 0, 0
        start = self.global_step
        for _ in tqdm(range(total), disable=not self.dist.is_main, leave=False):
            topo = self.topo_index[self.env.current_network]
            with trace_range("act"):
                action = self.post_process_actions(self._choose_action(self.obs, topo))
            with trace_range("sim"):
                next_obs, reward, done, _, _ = self.env.step(action)
            stats = self.env.current_simulator_state.network_stats
            succ += stats["run_successful_flows"]
            drop += stats["run_dropped_flows"]
            ep_ret += float(reward)
            self.rb.add(self._node_rows(self.obs).numpy(), topo, self._node_rows(next_obs).numpy(), action, reward,
                        float(done))
            self.sps.add(1)
            self.obs = next_obs
            if done:
                self.episode += 1
                self._episode_end(ep_ret, {"charts/success_ratio": succ / max(succ + drop, 1)})
                ep_ret, succ, drop = 0.0, 0, 0
                self.obs, _ = self.env.reset(seed=h.seed)  # AutoResetWithSeed: same seed every episode
            # reference simple_ddpg.py:308 trains at the episode end once global_step >= warm-up - 1
            if (self.global_step % self.episode_steps == self.episode_steps - 1
                    and self.global_step >= self.warmup - 1):
                with trace_range("learn"):
                    for _ in range(self.episode_steps):
                        self.learner.update(self.rb.sample(self.batch_size, self.device))
                self.metrics.log({f"losses/{k}": float(v) for k, v in self.learner.last.items()}, self.global_step)
            self.global_step += 1
        return {"steps": self.global_step - start, "episodes": self.episode, "best_return": self.best_return}

    def _train_batched(self, episodes: int) -> dict:
        tr = self.trainer
        total = episodes * self.episode_steps
        start = self.global_step
        for _ in tqdm(range(total), disable=not self.dist.is_main, leave=False):
            tr.step()
            self.global_step = tr.global_step
            self.sps.add(self.num_envs * self.dist.world_size)
            if tr.global_step % self.episode_steps == 0:
                self.episode = tr.episode
                m = tr.metrics(reset=True)
                info = {"charts/success_ratio": m["success_ratio"], "charts/episodes_finished": m["episodes"]}
                info.update({f"losses/{k}": m[k] for k in ("qf1_loss", "actor_loss", "qf1_values") if k in m})
                self._episode_end(m["mean_episode_return"], info)
        tr.flush()   # the caller's stream waits for the trainer's streams before anything reads their results
        self.sim.check_flags()
        return {"steps": self.global_step - start, "episodes": self.episode, "best_return": self.best_return}

    # ------------------------------------------------------------------------------------------
    # testing (reference main.py:53-76 — greedy episode on the inference network, simulator CSVs)
    def test(self, episode_steps: Optional[int] = None, seed: Optional[int] = None) -> dict:
        env = self._make_env(test_mode=True)
        h = self.agent_helper
        obs, _ = env.reset(seed=h.seed if seed is None else seed)
        topo = self.topo_index.get(env.current_network, self.topo_index[h.schedule["inference_network"]])
        steps = int(episode_steps or self.episode_steps)
        total_r, succ, drop = 0.0, 0, 0
        for _ in range(steps):
            action = self.predict(obs, topo)
            obs, reward, done, _, _ = env.step(action)
            st = env.current_simulator_state.network_stats
            succ += st["run_successful_flows"]
            drop += st["run_dropped_flows"]
            total_r += float(reward)
            if done:
                break
        env.close()
        return {"return": total_r, "success_ratio": succ / max(succ + drop, 1), "succ": succ, "drop": drop}

    # ------------------------------------------------------------------------------------------
    # persistence
    def save_actor(self, path: str) -> None:
        if self.dist.is_main:
            ckpt.save_actor(path, self.actor, self.cfg, self.n_obs, self.action_dim, self.n_pad, self.C, self.F)

    def load_actor_weights(self, path: str) -> None:
        d = torch.load(path, map_location="cpu", weights_only=True)
        if d.get("format") != ckpt.ACTOR_FORMAT:
            raise ValueError(f"{path}: not an actor file")
        if self.backend == "batched":
            self.trainer.flush()  # in-flight steps finish before the weights change; the next step re-syncs
        self.actor.load_state_dict(d["state_dict"])
        self.learner.target_actor.load_state_dict(d["state_dict"])
        self.learner.refresh_shadows()

    def state_dict(self) -> dict:
        base = {"backend": self.backend, "global_step": self.global_step, "episode": self.episode,
                "best_return": float(self.best_return)}
        if self.backend == "batched":
            # the replay ring is checkpointed when it is small enough (exact resume); a multi-GB ring
            # (millions of transitions) is skipped unless checkpoint_replay="yes" — resume then refills it
            pol = self.checkpoint_replay
            rb = self.trainer.replay_bytes()
            keep = pol == "yes" or (pol == "auto" and rb <= self.checkpoint_replay_max)
            if not keep:
                logger.info(f"checkpoint without the replay ring ({rb / 2**30:.1f} GiB)")
            base["trainer"] = self.trainer.state_dict(include_replay=keep)
        else:
            n = len(self.rb)
            base["learner"] = self.learner.state_dict()
            base["replay"] = {"pos": self.rb.pos, "full": self.rb.full,
                              **{k: torch.from_numpy(getattr(self.rb, k)[:n].copy())
                                 for k in ("obs", "next_obs", "topo", "actions", "rewards", "dones")}}
            name, keys, pos, has_gauss, cached = self.rb.rng.get_state()
            base["rng"] = {"explore": self.np_rng.bit_generator.state,
                           "replay": {"keys": torch.from_numpy(keys.astype(np.int64)), "pos": int(pos),
                                      "has_gauss": int(has_gauss), "cached": float(cached)}}
        return base

    def load_state_dict(self, sd: dict) -> None:
        if sd["backend"] != self.backend:
            raise ValueError(f"checkpoint backend {sd['backend']} != {self.backend}")
        self.global_step, self.episode = int(sd["global_step"]), int(sd["episode"])
        self.best_return = float(sd["best_return"])
        if self.backend == "batched":
            self.trainer.load_state_dict(sd["trainer"])
        else:
            self.learner.load_state_dict(sd["learner"])
            r = sd["replay"]
            n = r["obs"].shape[0]
            for k in ("obs", "next_obs", "topo", "actions", "rewards", "dones"):
                getattr(self.rb, k)[:n] = r[k].numpy()
            self.rb.pos, self.rb.full = int(r["pos"]), bool(r["full"])
            self.np_rng.bit_generator.state = sd["rng"]["explore"]
            rr = sd["rng"]["replay"]
            self.rb.rng.set_state(("MT19937", rr["keys"].numpy().astype(np.uint32), rr["pos"], rr["has_gauss"],
                                   rr["cached"]))
            if self.env is not None:  # resume at an episode boundary: same-seed reset of the right network
                self.env.close()
                self.env = None
        # keep replicas identical after a resume
        from gsc_amd.parallel.dist import broadcast_tensors
        L = self.learner
        if self.dist.enabled:
            broadcast_tensors([L.actor_flat.flat, L.critic_flat.flat, L.target_actor_flat.flat,
                               L.target_critic_flat.flat])
        L.refresh_shadows()

    def _per_rank(self) -> bool:
        return self.backend == "batched" and self.dist.world_size > 1

    def save_checkpoint(self, path: str) -> None:
        """Rank 0 writes ``path`` (learner + its trainer state).  Data parallel: every other rank writes
        its own simulator states / replay ring / RNG state to ``ckpt.rank_path(path, r)`` -- the shards
        are rank-seeded and must stay disjoint after a resume.  Every file of one save carries the same
        stamp (global step, episode, world size), and the ranks meet at a barrier once all are written,
        so a save interrupted between two ranks' writes is detected on resume."""
        sd = self.state_dict()
        nonce = ckpt.new_nonce()
        if self._per_rank():
            from gsc_amd.parallel.dist import sync_string
            nonce = sync_string(nonce)  # rank 0's: one stamp for every file of this save
        stamp = ckpt.save_stamp(sd, self.dist.world_size, nonce)
        meta = {"experiment_id": self.agent_helper.experiment_id, "time": time.time(), "rank": self.dist.rank,
                "world_size": self.dist.world_size, "stamp": stamp}
        if self._per_rank() and self.dist.rank > 0:
            sd["trainer"].pop("learner", None)       # replicas are identical: rank 0's file holds the learner
            ckpt.save_checkpoint(ckpt.rank_path(path, self.dist.rank), sd, meta=meta, rank=0)
        else:
            ckpt.save_checkpoint(path, sd, meta=meta, rank=self.dist.rank)
        if self._per_rank():
            from gsc_amd.parallel.dist import barrier
            barrier()

    def load_checkpoint(self, path: str) -> None:
        d0 = ckpt.load_checkpoint(path)
        sd = d0["state"]
        if self._per_rank() and self.dist.rank > 0:
            rp = ckpt.rank_path(path, self.dist.rank)
            stamp = d0.get("meta", {}).get("stamp") or {}
            why = "missing"
            if os.path.exists(rp):
                dr = ckpt.load_checkpoint(rp)
                # stamps written before the per-save nonce existed have none: compare them as nonce ''
                got = dict(dr.get("meta", {}).get("stamp") or {})
                got.setdefault("nonce", "")
                stamp = dict(stamp)
                stamp.setdefault("nonce", "")
                want = ckpt.save_stamp(sd, self.dist.world_size, stamp["nonce"])
                if got == stamp and stamp == want:
                    local = dr["state"]
                    local["trainer"]["learner"] = sd["trainer"]["learner"]
                    self.load_state_dict(local)
                    return
                why = f"from another save (stamp {got} != rank 0's {stamp})"
            # no matching per-rank state (fewer ranks, or a save interrupted between two ranks' writes):
            # take rank 0's learner, drop rank 0's replay ring (this rank's shard must not start as a copy
            # of rank 0's transitions: it refills with a full warm-up) and re-seed this rank's simulator
            # streams / replay sampler so the shards stay disjoint
            logger.warning(f"{rp} {why}: rank {self.dist.rank} re-seeds its simulator and replay sampler and "
                           "refills its replay ring")
            sd["trainer"].pop("replay", None)
            self.load_state_dict(sd)
            self.trainer.reseed(int(self.agent_helper.seed) * 1000 + self.dist.rank)
            return
        self.load_state_dict(sd)

    def close(self) -> None:
        if self.rewards_writer is not None:
            self.rewards_writer.close()
        self.metrics.close()
        if self.backend == "oracle" and self.env is not None:
            self.env.close()
