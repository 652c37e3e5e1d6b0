"""HIP-graph capture of a whole single-GPU training step (forward, loss, backward, fused
optimizer step).

At small per-GPU batches (the reference trains with 16-128 images per process,
BASELINE/main.py:30, CDR/train.sh:4, NESTED/train.py:470) a ResNet-50 step is ~600 kernel
launches of a few microseconds each and the host launch path, not the GPU, sets the step
time.  Capturing the step once and replaying it issues the whole dependency chain with one
``hipGraphLaunch``.  Every op of the step is capture-safe: no host synchronisation, device
tables (optimizer / weight-prep) built once and cached, outputs from the caching allocator's
graph pool.

Constraints (checked or documented): inputs and labels must live in the static tensors the
step closes over (copy new batches into them); hyper-parameters baked into kernel arguments
(the learning rate) are those at capture time -- recapture after changing them.  Multi-process
steps are capturable with this framework's bucket engine (parallel/reducer.py: its packing,
all-reduces, per-bucket optimizer and the SyncBN collectives are all stream-ordered launches);
torch's DistributedDataParallel Reducer is not.

Host-side counters: a replay runs no Python, so counters the step advances on the host --
BatchNorm2d's pending ``num_batches_tracked`` and FusedAdam's ``state["step"]`` -- would
freeze at their capture-time values.  :class:`HostCounters` records what the captured call
advanced and re-applies it after every replay (Adam's bias correction itself reads a device
counter the captured step increments, optim/fused.py).
"""
from __future__ import annotations

import os

import torch


def _stale_weights():
    """Mark every cached bf16 weight copy stale before a capture.  Which kernels the captured
    step contains is decided by host-side state at capture time: a capture right after an
    evaluation pass (weights fresh) would record no weight-prep launch, and every replay --
    each ending in an optimizer step -- would then run on the pre-capture bf16 weights."""
    from ..ops import functional as Fn

    Fn.bump_weight_generation()


class HostCounters:
    """Per-replay host bookkeeping of a captured step: the BN ``_nbt_pending`` increments the
    capture recorded (module by module) plus each optimizer's ``on_graph_replay`` hook."""

    def __init__(self, modules=(), optimizers=()):
        seen, self.bns = set(), []
        for r in modules:
            for m in r.modules():
                if hasattr(m, "_nbt_pending") and id(m) not in seen:  # a module reachable twice counts once
                    seen.add(id(m))
                    self.bns.append(m)
        self.opts = [o for o in optimizers if hasattr(o, "on_graph_replay")]
        self.before = self.delta = None

    def begin_capture(self):
        self.before = [m._nbt_pending for m in self.bns]

    def end_capture(self):
        self.delta = [m._nbt_pending - b for m, b in zip(self.bns, self.before)]

    def replayed(self):
        for m, d in zip(self.bns, self.delta or ()):
            m._nbt_pending += d
        for o in self.opts:
            o.on_graph_replay()


def _capture_mode():
    """With a process group, capture thread-locally: the RCCL process group's watchdog thread polls
    the HIP events of collectives issued before the capture (the warm-up steps' all-reduces), and a
    global-mode capture turns any such query from another thread into a capture error.  Stream
    capture itself is per stream, so the kernels and collectives the autograd device thread issues
    on the capturing streams are captured either way; what thread-local mode gives up is HIP's
    unsafe-call check in threads other than the capturing one."""
    return "thread_local" if torch.distributed.is_initialized() else "global"


def _check_capture_safe_pg():
    """Before a capture with an RCCL process group: the group must have been created with its CUDA
    event cache off (``parallel.ddp.graph_safe_nccl_env()`` before ``init_process_group``).  With
    the cache on, a collective captured into the graph re-records a cached event object that the
    watchdog may still be polling for an older, eager work; HIP refuses that query with
    hipErrorCapturedEvent and the watchdog aborts the process (the intermittent abort of
    tests/test_ddp_gpu.py::test_bench_force_ddp_rccl_world1[True] in round 4).  With fresh events
    per work no event the watchdog polls is ever recorded inside a capture, and the captured works
    themselves never reach the watchdog's list.

    That alone is not enough (round 5: the same abort in
    test_main_graph_force_ddp_side_stream_matches_eager, at the recapture after an epoch's eager
    validation collectives): a capture that issues a collective makes the group's RCCL stream join
    the capture, and HIP refuses a query of ANY event last recorded on that stream -- including
    the end event of an eager work the watchdog has not yet retired (it sweeps its list every
    ~100 ms).  So before the capture every eager work must have left every group's watchdog list:
    ``_wait_for_pending_works`` returns exactly when the list is empty, an observable condition
    instead of a sleep."""
    if not torch.distributed.is_initialized() or torch.distributed.get_backend() != "nccl":
        return
    if os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE", "1") not in ("0", "false", "False"):
        raise RuntimeError("HIP-graph capture with an RCCL process group needs TORCH_NCCL_CUDA_EVENT_CACHE=0 at "
                           "process-group creation: call parallel.ddp.graph_safe_nccl_env() before "
                           "init_process_group (bench.py --graph and main.py --graph do)")
    torch.cuda.synchronize()
    drain_rccl_watchdogs()


def drain_rccl_watchdogs():
    """Block until the watchdog of every RCCL process group (the default group, the SyncBN group,
    any subgroup) has retired all its eager works (call after a device synchronize, so they are
    complete; the wait is then at most one watchdog sweep)."""
    from torch.distributed import distributed_c10d as c10d

    for pg in list(c10d._world.pg_map):
        try:
            if c10d.get_backend(pg) != "nccl":
                continue
        except (RuntimeError, ValueError):
            continue
        pg._wait_for_pending_works()


class GraphedStep:
    """``GraphedStep(step_fn, warmup=3)``: runs ``step_fn`` ``warmup`` times on a side stream
    (allocator / autograd / table warm-up), captures one call, then ``__call__`` replays it and
    returns the captured step's output tensors (overwritten by every replay)."""

    def __init__(self, step_fn, warmup: int = 3, device=None, counters: HostCounters = None,
                 distributed: bool = False):
        if torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1 and not distributed:
            raise RuntimeError("GraphedStep: a multi-process step is capturable only through the bucket engine "
                               "(pass distributed=True for a GradSyncDDP model; torch DDP's reducer is not)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                step_fn()
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        _check_capture_safe_pg()
        _stale_weights()
        self.counters = counters
        if counters is not None:
            counters.begin_capture()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode=_capture_mode()):
            self.out = step_fn()
        if counters is not None:
            counters.end_capture()
        self.replays = 0

    def __call__(self):
        self.graph.replay()
        # the first replay executes the step whose host side effects the capture already made
        if self.replays and self.counters is not None:
            self.counters.replayed()
        self.replays += 1
        return self.out


class StepGrapher:
    """Graph the training step of a data loop: ``grapher(*batch)`` runs the first ``warmup``
    steps eagerly (side stream), captures the step on the next call and replays it (the capture
    itself executes nothing, so that batch is trained by the first replay); later calls copy the
    batch into the captured static inputs and replay.  A batch of a different shape (the short
    last batch of an epoch) runs eagerly.  Call :meth:`reset` after changing anything baked into
    the captured kernels' arguments (the learning rate at an epoch boundary): the next call
    recaptures.  Every step -- eager, captured or replayed -- trains on exactly one batch."""

    def __init__(self, step_fn, warmup: int = 2, counters: HostCounters = None):
        self.fn, self.warmup, self.calls = step_fn, max(1, warmup), 0
        self.graph = self.static = self.out = None
        self.captures = 0
        self.counters = counters

    def reset(self):
        self.graph = self.static = self.out = None
        self.calls = 0  # eager warm-up again before the next capture

    def eager(self, *tensors):
        """One eager step on a side stream (steps that must not be captured: LR warm-up)."""
        return self._eager(tensors)

    def _eager(self, tensors):
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            out = self.fn(*tensors)
        cur.wait_stream(side)
        return out

    def __call__(self, *tensors):
        self.calls += 1
        if self.calls <= self.warmup:
            return self._eager(tensors)
        if self.graph is not None and any(s.shape != t.shape or s.dtype != t.dtype
                                          for s, t in zip(self.static, tensors)):
            return self._eager(tensors)
        if self.graph is None:
            torch.cuda.synchronize()
            _check_capture_safe_pg()
            _stale_weights()
            self.static = [t.clone() for t in tensors]
            if self.counters is not None:
                self.counters.begin_capture()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode=_capture_mode()):
                self.out = self.fn(*self.static)
            if self.counters is not None:
                self.counters.end_capture()
            self.captures += 1
        else:
            for s, t in zip(self.static, tensors):
                s.copy_(t, non_blocking=True)
            if self.counters is not None:
                self.counters.replayed()  # the capture call itself made the first replay's host effects
        self.graph.replay()
        return self.out
