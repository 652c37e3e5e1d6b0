"""Checkpoint / resume.

The reference pickles the whole DDP module on EVERY rank into the same file
each epoch (BASELINE/main.py:308-310, a write race) and cannot resume;
NESTED saves best-only ``{'feat','cls'}`` state_dicts (NESTED/train.py:154-161)
and ``--resumePth`` reloads weights only (:372-378).

Here: rank 0 writes a ``state_dict`` checkpoint (unwrapped model(s),
optimizer(s), scheduler(s), epoch/step, RNG states, config, metrics) to a
temp file and atomically renames it; every rank waits on a barrier.
``last.pth`` every epoch, ``best.pth`` on improvement; :func:`load_checkpoint`
restores all of it (``weights_only=True`` is used for anything not written by
this framework).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
import torch.distributed as dist

from ..ops import functional as Fn


def _unwrap(m):
    from ..parallel.reducer import GradSyncDDP

    return m.module if isinstance(m, (torch.nn.parallel.DistributedDataParallel, GradSyncDDP)) else m


def rng_state():
    name, keys, pos, has_gauss, cached = np.random.get_state()
    st = {"python": random.getstate(), "numpy": (name, torch.from_numpy(keys.astype(np.int64)), int(pos),
                                                 int(has_gauss), float(cached)),
          "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st):
    py = st["python"]
    random.setstate((py[0], tuple(py[1]), py[2]))
    name, keys, pos, has_gauss, cached = st["numpy"]
    np.random.set_state((name, keys.numpy().astype(np.uint32), pos, has_gauss, cached))
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        try:
            torch.cuda.set_rng_state_all(st["cuda"])
        except Exception:
            pass


def is_rank0():
    return not dist.is_initialized() or dist.get_rank() == 0


def barrier():
    if dist.is_initialized():
        dist.barrier()


def _world():
    return dist.get_world_size() if dist.is_initialized() else 1


def save_checkpoint(path, models: dict, optimizers: dict = None, schedulers: dict = None, **extra):
    """Rank-0 atomic write; all ranks sync on a barrier afterwards.  Every rank's RNG
    state is gathered into the file (ranks are seeded seed+rank, so their augmentation /
    dropout / nested-K streams differ) and :func:`load_checkpoint` restores each rank's own."""
    per_rank = None
    if _world() > 1:
        per_rank = [None] * _world()
        dist.all_gather_object(per_rank, rng_state())
    if is_rank0():
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        state = {"models": {k: _unwrap(m).state_dict() for k, m in models.items()},
                 "optimizers": {k: o.state_dict() for k, o in (optimizers or {}).items()},
                 "schedulers": {k: s.state_dict() for k, s in (schedulers or {}).items()},
                 "rng": rng_state(), "format": "dcp-ckpt-v1"}
        if per_rank is not None:
            state["rng_per_rank"] = per_rank
        state.update(extra)
        tmp = f"{path}.tmp.{os.getpid()}"
        torch.save(state, tmp)
        os.replace(tmp, path)
    barrier()


def load_checkpoint(path, models: dict, optimizers: dict = None, schedulers: dict = None, map_location="cpu",
                    restore_rng=True, strict=True):
    state = torch.load(path, map_location=map_location, weights_only=True)
    if state.get("format") != "dcp-ckpt-v1":
        # plain state_dict (e.g. NESTED netBest.pth {'feat','cls'} or a bare model state_dict)
        if "feat" in state and "cls" in state and "feat" in models:
            feat = _unwrap(models["feat"])
            sd = state["feat"]
            if hasattr(feat, "net") and not any(k.startswith("net.") for k in sd):
                # a reference-trained NetFeat (feat_net.* / conv2_x names): onto our NetFeat.net
                from ..models.pretrained import remap_reference_keys

                sd = {"net." + k: v for k, v in remap_reference_keys(sd).items()}
            feat.load_state_dict(sd, strict=strict)
            _unwrap(models["cls"]).load_state_dict(state["cls"], strict=strict)
        else:
            next(iter(models.values())).load_state_dict(state, strict=strict)
        Fn.bump_weight_generation()
        return {}
    for k, m in models.items():
        if k in state["models"]:
            _unwrap(m).load_state_dict(state["models"][k], strict=strict)
    for k, o in (optimizers or {}).items():
        if k in state["optimizers"]:
            o.load_state_dict(state["optimizers"][k])
    for k, s in (schedulers or {}).items():
        if k in state["schedulers"]:
            s.load_state_dict(state["schedulers"][k])
    if restore_rng:
        per_rank = state.get("rng_per_rank")
        rank = dist.get_rank() if dist.is_initialized() else 0
        if per_rank is not None and len(per_rank) == _world():
            set_rng_state(per_rank[rank])
        elif "rng" in state and _world() == 1:
            set_rng_state(state["rng"])
        # a different world size than the one that wrote the file: keep this rank's own
        # (seed + rank) stream rather than giving every rank rank 0's
    Fn.bump_weight_generation()
    return {k: v for k, v in state.items() if k not in ("models", "optimizers", "schedulers", "rng", "rng_per_rank")}
