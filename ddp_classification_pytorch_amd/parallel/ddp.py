"""Data parallelism over RCCL (torch.distributed backend "nccl" = RCCL on ROCm).

Reference: one process per GPU, ``SyncBatchNorm.convert_sync_batchnorm`` +
``DistributedDataParallel(device_ids=[local_rank])`` (BASELINE/main.py:147-149,
ARCFACE/arc_main.py:238-243).

MI355X choices:
* 25 MB gradient buckets with a small first bucket.  ResNet-50's grads are
  97.5 MB fp32 and most of them sit in layer4, whose gradients are ready
  first.  A 100 MB cap leaves one 89.7 MB bucket that can only start after
  the stem's wgrad, fully exposed after backward.  25 MB gives
  [7.8, 30.0, 25.0, 25.3, 9.3] MB: the first four overlap the backward of
  layers 3..1, and only the 9.3 MB tail (~0.1 ms per xGMI ring) is exposed;
* ``gradient_as_bucket_view=True`` (no grad->bucket copies);
* ``broadcast_buffers=False``: BN running stats are either identical by
  construction (SyncBN) or rank-local (local BN), so the per-forward buffer
  broadcast the reference pays (C3) is skipped;
* SyncBN is our fused BN with a ``process_group``: one packed all_reduce of
  (sum, sumsq) per layer forward, one of (sum dz, sum dz*xhat) backward.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.layers import BatchNorm2d


def init_distributed(backend: str = None, timeout_s: int = 1800):
    """torchrun / torch.distributed.launch compatible init.  Returns (rank, local_rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    return rank, local, world


def convert_sync_batchnorm(model: nn.Module, process_group=None) -> nn.Module:
    """Attach a process group to every fused BatchNorm2d (in place)."""
    group = process_group if process_group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    for m in model.modules():
        if isinstance(m, BatchNorm2d):
            m.process_group = group
    return model


def wrap_ddp(model: nn.Module, local_rank: int = None, syncbn: bool = False, bucket_cap_mb: float = 25.0,
             first_bucket_mb: float = 4.0, find_unused: bool = False, static_graph: bool = False):
    if syncbn:
        convert_sync_batchnorm(model)
    if not dist.is_initialized() or dist.get_world_size() == 1 and not syncbn:
        return model
    kw = dict(broadcast_buffers=False, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
              find_unused_parameters=find_unused, static_graph=static_graph)
    if next(model.parameters()).is_cuda:
        kw["device_ids"] = [local_rank if local_rank is not None else torch.cuda.current_device()]
    # first bucket size: read by the DDP constructor (torch/nn/parallel/distributed.py:1204,1242-1245)
    prev = getattr(dist, "_DEFAULT_FIRST_BUCKET_BYTES", None)
    dist._DEFAULT_FIRST_BUCKET_BYTES = int(first_bucket_mb * 1024 * 1024)
    try:
        ddp = nn.parallel.DistributedDataParallel(model, **kw)
    finally:
        if prev is not None:
            dist._DEFAULT_FIRST_BUCKET_BYTES = prev
    return ddp


def unwrap(model: nn.Module) -> nn.Module:
    return model.module if isinstance(model, nn.parallel.DistributedDataParallel) else model


@torch.no_grad()
def all_reduce_metrics(vec: torch.Tensor, op=None) -> torch.Tensor:
    """Exact distributed metrics: one all_reduce of a packed vector (loss sum, correct@1, correct@3, count)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(vec, op=op or dist.ReduceOp.SUM)
    return vec


def reduce_loss(loss: torch.Tensor, world_size: int) -> torch.Tensor:
    """BASELINE/main.py:52-56: reduce to rank 0 and average there."""
    t = loss.detach().clone()
    if dist.is_initialized() and world_size > 1:
        dist.reduce(t, dst=0)
        if dist.get_rank() == 0:
            t /= world_size
    return t
