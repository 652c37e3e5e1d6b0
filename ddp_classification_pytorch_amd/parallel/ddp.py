"""Data parallelism over RCCL (torch.distributed backend "nccl" = RCCL on ROCm).

Reference: one process per GPU, ``SyncBatchNorm.convert_sync_batchnorm`` +
``DistributedDataParallel(device_ids=[local_rank])`` (BASELINE/main.py:147-149,
ARCFACE/arc_main.py:238-243).

MI355X choices:
* 25 MiB gradient buckets with a 4 MiB first bucket.  ResNet-50's grads are
  97.5 MB fp32 and most of them sit in layer4, whose gradients are ready
  first.  A 100 MB cap leaves one 89.7 MB bucket that can only start after
  the stem's wgrad, fully exposed after backward.  With 25 MiB buckets the
  all-reduces of layer4..layer2 overlap the backward of the layers below,
  and only the last (layer1 + stem side) bucket is exposed; the small first
  bucket starts the first all-reduce as soon as the head/layer4 tail
  gradients exist.  The layout is pinned by tests/test_ddp_buckets_cpu.py
  from the Reducer itself (``bucket_layout_mb``);
* ``gradient_as_bucket_view=True`` (no grad->bucket copies);
* ``broadcast_buffers=False``: BN running stats are either identical by
  construction (SyncBN) or rank-local (local BN), so the per-forward buffer
  broadcast the reference pays (C3) is skipped;
* SyncBN is our fused BN with a ``process_group``: forward all-gathers each rank's
  per-channel (n, mean, M2) and Chan-merges them (the forward statistics are exact for any
  per-rank counts), backward all-reduces (sum g, sum g*xhat) and normalises them by
  ``per-rank count x world``: the backward assumes EQUAL per-rank batches, which the
  rank-sharded sampler guarantees (it pads every rank to the same number of samples, so every
  step's per-rank batch is the same; ``DCP_SYNCBN_CHECK=1`` verifies the gathered counts at every
  SyncBN forward, at the price of a host sync per layer); a projection block's two BNs share one
  collective in each direction.  Those collectives run on a DEDICATED process group
  (:func:`bn_process_group`: its own RCCL communicator and stream), so a 516 B..16 KB
  statistics exchange that sits on the critical path never queues behind a 25 MiB
  gradient bucket the Reducer has in flight on the default group.  Per ResNet-50
  step: 49 forward gathers + 49 backward reduces (53 BNs, 4 projection pairs).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.layers import BatchNorm2d


def graph_safe_nccl_env():
    """Call before init_process_group when steps will be captured into HIP graphs.  The RCCL
    process group's event cache hands a finished collective's events to the next collective; a
    captured collective records them inside the graph, and the watchdog thread's later query of
    such an event (from a work enqueued eagerly around the capture) fails with
    hipErrorCapturedEvent and aborts the process (seen intermittently in
    tests/test_ddp_gpu.py::test_bench_force_ddp_rccl_world1[True]).  Fresh events per collective
    cost a few microseconds each; only the graph path pays it."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init_distributed(backend: str = None, timeout_s: int = 1800, force: bool = False):
    """torchrun / torch.distributed.launch compatible init.  Returns (rank, local_rank, world).
    ``force``: create the process group at world size 1 too (``--force-ddp``: one process runs the
    data-parallel engine over a real, single-rank RCCL communicator)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    return rank, local, world


_BN_GROUPS = {}


def bn_process_group():
    """The SyncBN communicator: one extra group over all ranks, created once per default group
    (collectively: every rank calls this in the same order, from convert_sync_batchnorm).

    ``DCP_SYNCBN_SHARED_GROUP=1`` (``--syncbn-shared-group``): the default group instead -- the BN
    statistics collectives then share the gradient communicator and its stream, serialised with the
    bucket all-reduces in issue order (a statistics exchange can wait behind a 25 MiB bucket).  That
    is the fallback for stacks where two RCCL communicators in flight at once on one GPU (the BN
    group on the compute stream, the buckets on the side stream) could deadlock when kernel
    residency differs across ranks."""
    if not dist.is_initialized():
        return None
    if os.environ.get("DCP_SYNCBN_SHARED_GROUP", "0") == "1":
        return dist.group.WORLD
    key = id(dist.group.WORLD)
    g = _BN_GROUPS.get(key)
    if g is None:
        g = _BN_GROUPS[key] = dist.new_group(ranks=list(range(dist.get_world_size())))
    return g


def convert_sync_batchnorm(model: nn.Module, process_group=None, transport: str = None) -> nn.Module:
    """Attach a process group to every fused BatchNorm2d (in place); by default the dedicated
    SyncBN group (:func:`bn_process_group`), not the group the DDP Reducer all-reduces on.
    ``transport``: "rccl" (default; ``DCP_SYNCBN_TRANSPORT``) or "peer" -- the statistics
    collectives through the IPC-mapped mailboxes of :mod:`parallel.peer` (one kernel per exchange,
    collective setup; falls back to RCCL where a peer cannot be mapped)."""
    group = process_group if process_group is not None else bn_process_group()
    for m in model.modules():
        if isinstance(m, BatchNorm2d):
            m.process_group = group
    transport = transport or os.environ.get("DCP_SYNCBN_TRANSPORT", "rccl")
    if transport not in ("rccl", "peer"):
        raise ValueError(f"unknown SyncBN transport {transport!r} (rccl | peer)")
    if group is not None and torch.cuda.is_available():
        from . import peer

        if transport == "peer":
            peer.enable(group)
        else:
            peer.disable(group)
    return model


DEFAULT_ENGINE = os.environ.get("DCP_DDP_ENGINE", "dcp")


def wrap_ddp(model: nn.Module, local_rank: int = None, syncbn: bool = False, bucket_cap_mb: float = 25.0,
             first_bucket_mb: float = 4.0, find_unused: bool = False, static_graph: bool = False,
             force: bool = False, engine: str = None, comm_dtype=torch.float32, telemetry: bool = False):
    """Data parallelism over the default group (RCCL on GPU, gloo on CPU).

    ``engine="dcp"`` (default; ``DCP_DDP_ENGINE``): this framework's bucket engine
    (:class:`parallel.reducer.GradSyncDDP`): graph-capturable, optimizer fusable per bucket
    (:func:`attach_optimizer`), bf16 all-reduce with ``comm_dtype=torch.bfloat16``.
    ``engine="torch"``: torch's ``DistributedDataParallel`` (C++ Reducer), configured as below.

    Bucket limits: torch's Reducer honours a separate first-bucket limit only when the
    DDP constructor sees ``bucket_cap_mb=None`` (its 25 MiB default,
    torch/nn/parallel/distributed.py:828-834, 1242-1247); an explicit cap is used for the
    first bucket too.  So the default 25 MiB cap is passed as ``None`` with
    ``dist._DEFAULT_FIRST_BUCKET_BYTES`` set for the constructor, and any other cap gives
    uniform buckets.  ``bucket_layout_mb`` reports what was actually built.
    ``force``: wrap even at world size 1 (tests)."""
    if syncbn:
        convert_sync_batchnorm(model)
    if not force and (not dist.is_initialized() or dist.get_world_size() == 1 and not syncbn):
        return model
    engine = engine or DEFAULT_ENGINE
    if engine == "dcp":
        if find_unused:
            raise ValueError("the dcp bucket engine needs every parameter used (find_unused=False)")
        from .reducer import GradSyncDDP

        return GradSyncDDP(model, None, bucket_cap_mb, first_bucket_mb, comm_dtype, telemetry)
    if engine != "torch":
        raise ValueError(f"unknown DDP engine {engine!r} (dcp | torch)")
    default_cap = abs(float(bucket_cap_mb) - 25.0) < 1e-9
    kw = dict(broadcast_buffers=False, bucket_cap_mb=None if default_cap else bucket_cap_mb,
              gradient_as_bucket_view=True, find_unused_parameters=find_unused, static_graph=static_graph)
    if next(model.parameters()).is_cuda:
        kw["device_ids"] = [local_rank if local_rank is not None else torch.cuda.current_device()]
    prev = getattr(dist, "_DEFAULT_FIRST_BUCKET_BYTES", None)
    if default_cap and first_bucket_mb:
        dist._DEFAULT_FIRST_BUCKET_BYTES = int(first_bucket_mb * 1024 * 1024)
    try:
        ddp = nn.parallel.DistributedDataParallel(model, **kw)
    finally:
        if prev is not None:
            dist._DEFAULT_FIRST_BUCKET_BYTES = prev
    return ddp


def attach_optimizer(net: nn.Module, opt):
    """Fuse ``opt``'s step into the bucket engine (one launch per bucket behind its all-reduce);
    a no-op for torch DDP and unwrapped (single-process) models."""
    if hasattr(net, "reducer") and hasattr(net, "attach_optimizer"):
        net.attach_optimizer(opt)
    return opt


def bucket_layout_mb(ddp: nn.Module):
    """Gradient bucket sizes (MiB, in all-reduce order) of a DDP module's Reducer.  The
    layout is final after the first backward (DDP rebuilds buckets in gradient-ready order)."""
    if hasattr(ddp, "reducer") and hasattr(ddp.reducer, "bucket_sizes_mb"):
        return ddp.reducer.bucket_sizes_mb()
    data = ddp._get_ddp_logging_data()
    sizes = data.get("rebuilt_bucket_sizes") or data.get("bucket_sizes", "")
    if isinstance(sizes, str):
        sizes = [int(v) for v in sizes.split(",") if v.strip()]
    return [v / 2**20 for v in sizes]


def unwrap(model: nn.Module) -> nn.Module:
    from .reducer import GradSyncDDP

    return model.module if isinstance(model, (nn.parallel.DistributedDataParallel, GradSyncDDP)) else model


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
