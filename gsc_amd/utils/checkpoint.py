"""Checkpoint / resume.

Reference: ``main.py:47-50`` pickles the whole ``Actor`` module to
``trained_actor.pt`` and the ``AgentHelper`` to ``agent_helper.obj``; nothing else is saved and
``--weights`` is parsed but never loaded.

Here every file loads with ``torch.load(..., weights_only=True)`` or ``json`` — nothing is
unpickled:

* ``trained_actor.pt`` — ``{"format", "agent_config", "obs_dim", "action_dim", "n_pad", "C", "F",
  "state_dict"}``; :func:`load_actor` rebuilds the :class:`~gsc_amd.models.Actor` from it.
* ``agent_helper.obj`` — JSON (:meth:`AgentHelper.to_json`).
* ``checkpoint.pt`` — full training state (actor, critic, both targets, Adam moments, replay ring,
  simulator state blobs, RNG states, global step / episode).  Rank 0 writes (atomically: temp
  file + rename); data parallel, rank r > 0 also writes its rank-local trainer state (simulator
  states, replay ring, sampler RNG -- all rank-seeded) to ``checkpoint.rank{r}.pt``.  On resume
  every rank loads the learner from rank 0's file plus its own rank-local state, and the learner
  re-broadcasts from rank 0, so replicas stay bit-identical and the env/replay shards disjoint.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

ACTOR_FORMAT = "gsc_amd.actor/1"
# /2: MLP matrices of the flat parameter buffers padded to 8 elements, trainer "rng" = the 5-int64
# device sampler state, per-rank files stamped with the save's (global_step, episode, world_size)
CHECKPOINT_FORMAT = "gsc_amd.checkpoint/2"
_OLD_FORMATS = {"gsc_amd.checkpoint/1": "flat parameter layout and sampler state changed in /2"}


def atomic_save(obj, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.realpath(path)), exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_actor(path: str, actor, agent_config: dict, obs_dim: int, action_dim: int, n_pad: int, C: int,
               F: int) -> None:
    sd = {k: v.detach().cpu().clone() for k, v in actor.state_dict().items()}
    atomic_save({"format": ACTOR_FORMAT, "agent_config": _plain(agent_config), "obs_dim": int(obs_dim),
                 "action_dim": int(action_dim), "n_pad": int(n_pad), "C": int(C), "F": int(F), "state_dict": sd},
                path)


def load_actor(path: str, device="cpu"):
    """-> (Actor in eval mode, header dict)."""
    from gsc_amd.models import Actor
    d = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(d, dict) or d.get("format") != ACTOR_FORMAT:
        raise ValueError(f"{path}: not a {ACTOR_FORMAT} file")
    actor = Actor(d["agent_config"], d["obs_dim"], d["action_dim"])
    actor.load_state_dict(d["state_dict"])
    actor.to(device).eval()
    return actor, {k: v for k, v in d.items() if k != "state_dict"}


def rank_path(path: str, rank: int) -> str:
    """File of rank ``rank``'s local trainer state (rank 0: ``path`` itself)."""
    if rank == 0:
        return path
    root, ext = os.path.splitext(path)
    return f"{root}.rank{rank}{ext}"


def save_checkpoint(path: str, state: dict, meta: Optional[dict] = None, rank: int = 0) -> None:
    if rank != 0:
        return
    atomic_save({"format": CHECKPOINT_FORMAT, "meta": _plain(meta or {}), "state": to_cpu(state)}, path)


def to_cpu(x):
    if torch.is_tensor(x):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(to_cpu(v) for v in x)
    return x


def load_checkpoint(path: str) -> dict:
    d = torch.load(path, map_location="cpu", weights_only=True)
    fmt = d.get("format") if isinstance(d, dict) else None
    if fmt in _OLD_FORMATS:
        raise ValueError(f"{path}: checkpoint format {fmt} is no longer readable ({_OLD_FORMATS[fmt]}); "
                         f"this build reads {CHECKPOINT_FORMAT}")
    if fmt != CHECKPOINT_FORMAT:
        raise ValueError(f"{path}: not a {CHECKPOINT_FORMAT} file")
    return d


def save_stamp(state: dict, world_size: int, nonce: str = "") -> dict:
    """Identity of one data-parallel save: every rank's file of the same save carries the same stamp.
    ``nonce`` (drawn by rank 0 and broadcast) tells apart two saves at the same step, e.g. a resumed run
    re-saving into the same directory next to a stale rank file."""
    return {"global_step": int(state["global_step"]), "episode": int(state["episode"]),
            "world_size": int(world_size), "nonce": str(nonce)}


def new_nonce() -> str:
    return os.urandom(8).hex()


def save_agent_helper(path: str, helper) -> None:
    with open(path, "w") as f:
        json.dump(_plain(helper.to_json()), f, indent=2, sort_keys=True)


def load_agent_helper(path: str):
    from gsc_amd.utils.experiment import AgentHelper
    with open(path) as f:
        return AgentHelper.from_json(json.load(f))


def _plain(x):
    """Reduce YAML/Python values to JSON-/weights_only-safe builtins."""
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, (str, int, float, bool)) or x is None:
        return x
    if hasattr(x, "item"):
        return x.item()
    return str(x)
