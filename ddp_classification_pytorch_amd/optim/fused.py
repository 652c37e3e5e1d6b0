"""Fused multi-tensor SGD / Adam on the gfx950 ``mt_sgd`` / ``mt_adam`` kernels.

Drop-in ``torch.optim.Optimizer`` subclasses (param groups, state_dict,
LR schedulers all work).  Semantics follow torch.optim.SGD / Adam exactly
(momentum buffer initialised to the first gradient; Adam bias correction;
L2 weight decay added to the gradient, or decoupled for AdamW), which the
reference uses at BASELINE/main.py:153 (SGD mom 0.9), ARCFACE/arc_main.py:249-253
(Adam / SGD wd 5e-4), NESTED/train.py:386-392 and PLC/utils.py:237 (nesterov).

GPU: one kernel launch per parameter group updates every tensor; the device
table of (param, grad, state) pointers is rebuilt only when a pointer changes.
CPU: the same math with torch ops (tests / gloo plumbing).

HIP-graph replay (engine/graph.py): a replayed step re-runs the captured kernels with
their captured arguments.  Adam's bias corrections therefore come from a device step
counter that the captured step itself increments (``mt_adam(step_dev=...)``), and
:meth:`FusedAdam.on_graph_replay` advances the host ``state["step"]`` mirrors so
``state_dict`` / resume see the true count.  SGD has no step-dependent argument; the
learning rate of a captured step is the one at capture (the grapher recaptures when it
changes).
"""
from __future__ import annotations

import math

import torch

from .. import _ext
from ..ops import functional as Fn

CHUNK = 4096


class _TableCache:
    """Device tables of one launch: the (param, grad, state..., numel) entries, rebuilt when a
    pointer changes (every eager step when grads are set to None), and the (entry, chunk) work
    list, which depends only on the tensor sizes and is built once (a per-step Python loop over
    ResNet-50's 6,240 chunks cost milliseconds of host time per eager step)."""

    def __init__(self):
        self.key = None
        self.sizes = None
        self.table = None
        self.chunks = None

    def get(self, entries, device):
        key = tuple((e[0], e[1], e[2], e[3], e[5]) for e in entries)
        if key != self.key:
            sizes = tuple(e[5] for e in entries)
            if sizes != self.sizes:
                counts = torch.tensor([(n + CHUNK - 1) // CHUNK for n in sizes], dtype=torch.int64)
                ent = torch.repeat_interleave(torch.arange(len(sizes), dtype=torch.int64), counts)
                first = torch.repeat_interleave(torch.cumsum(counts, 0) - counts, counts)
                ch = torch.stack([ent, torch.arange(ent.numel(), dtype=torch.int64) - first], 1)
                self.chunks = Fn.table_to_device(ch.to(torch.int32), torch.int32, device).view(-1, 2)
                self.sizes = sizes
            # graph-capture safe uploads (grads of a captured step live in the graph pool: the
            # table is rebuilt once during capture and replayed from the fill kernel's arguments)
            self.table = Fn.table_to_device([list(e) for e in entries], torch.int64, device).view(-1, 6)
            self.key = key
        return self.table, self.chunks


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 grad_scale=1.0):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, grad_scale=grad_scale)
        super().__init__(params, defaults)
        self._tables = {}
        self._fast = {}          # launch key -> (pointer fingerprint, table, chunks): see _update
        self._gid = None         # id(param) -> group index (step_params), rebuilt when groups change
        self._reducer_stepped = False

    def mark_stepped_by_reducer(self):
        """The bucket engine (parallel/reducer.py) already applied this step per bucket: the next
        ``step()`` is a no-op (the training loop's call after backward)."""
        self._reducer_stepped = True
        Fn.bump_weight_generation()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._fast.clear()  # new momentum buffers: the cached tables point at the old ones

    def _group_index(self):
        sig = tuple(len(g["params"]) for g in self.param_groups)
        if self._gid is None or self._gid[0] != sig:
            self._gid = (sig, {id(p): gi for gi, g in enumerate(self.param_groups) for p in g["params"]})
        return self._gid[1]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._reducer_stepped:
            self._reducer_stepped = False
            return loss
        self._step_subset(None)
        Fn.bump_weight_generation()
        return loss

    @torch.no_grad()
    def step_params(self, params):
        """Update only ``params`` (one bucket, right behind its all-reduce); every group's
        hyper-parameters apply to its own members.  The caller bumps the weight generation.
        Host cost is O(len(params)): the bucket's members are grouped by a cached param -> group
        map instead of scanning every group (the bucket engine calls this once per bucket)."""
        gid = self._group_index()
        by_group = {}
        for p in params:
            gi = gid.get(id(p))
            if gi is not None and p.grad is not None:
                by_group.setdefault(gi, []).append(p)
        for gi in sorted(by_group):
            self._step_group(gi, self.param_groups[gi], by_group[gi])

    def _step_subset(self, ids):
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None and (ids is None or id(p) in ids)]
            if params:
                self._step_group(gi, group, params)

    def _step_group(self, gi, group, params):
        mom = group["momentum"]
        # torch.optim.SGD initialises each momentum buffer to that parameter's first
        # gradient: parameters seen for the first time step with first=True in their own
        # launch, so a late-arriving gradient never resets the others' momentum
        fresh = set()
        for p in params:
            st = self.state[p]
            if mom != 0 and "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                fresh.add(p)
        for first, sub in ((True, [p for p in params if p in fresh]), (False, [p for p in params if p not in fresh])):
            if sub:
                self._update(gi, group, sub, first)

    def _update(self, gi, group, params, first):
        mom = group["momentum"]
        if params[0].is_cuda:
            # steady state: the parameters, their gradients (bucket views under the bucket engine)
            # and momentum buffers keep their addresses, so a pointer fingerprint of (param, grad)
            # stands in for rebuilding and comparing the whole table -- ~5x less host time per
            # step for ResNet-50 (momentum buffers only move on load_state_dict, which clears it)
            key = (gi, first, len(params), params[0].data_ptr())
            fp = tuple((p.data_ptr(), p.grad.data_ptr()) for p in params)
            hit = self._fast.get(key) if not first else None
            if hit is not None and hit[0] == fp:
                _ext.hip_ops().mt_sgd(hit[1], hit[2], group["lr"], mom, group["dampening"], group["weight_decay"],
                                      group["nesterov"], first, group["grad_scale"])
                return
            entries = []
            for p in params:
                if not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("FusedSGD needs contiguous params and grads")
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise RuntimeError("FusedSGD expects fp32 master params and grads")
                buf = self.state[p].get("momentum_buffer")
                entries.append((p.data_ptr(), p.grad.data_ptr(), buf.data_ptr() if buf is not None else 0, 0, 0,
                                p.numel()))
            key = (gi, first, len(params), params[0].data_ptr())  # one table per bucket subset
            table, chunks = self._tables.setdefault(key, _TableCache()).get(entries, params[0].device)
            if not first:
                self._fast[key] = (fp, table, chunks)
            _ext.hip_ops().mt_sgd(table, chunks, group["lr"], mom, group["dampening"], group["weight_decay"],
                                  group["nesterov"], first, group["grad_scale"])
            return
        for p in params:
            g = p.grad * group["grad_scale"]
            if group["weight_decay"]:
                g = g + group["weight_decay"] * p
            if mom:
                buf = self.state[p]["momentum_buffer"]
                if first:
                    buf.copy_(g)
                else:
                    buf.mul_(mom).add_(g, alpha=1 - group["dampening"])
                g = g + mom * buf if group["nesterov"] else buf
            p.add_(g, alpha=-group["lr"])


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False,
                 grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=decoupled,
                        grad_scale=grad_scale)
        super().__init__(params, defaults)
        self._tables = {}
        self._dsteps = {}        # launch key -> [device int32 step, host mirror, params]
        self._captured = None    # launch keys of the step being / last captured into a HIP graph
        self._reducer_stepped = False
        self._bucket_capture_open = False
        self._gid = None

    def mark_stepped_by_reducer(self):
        self._reducer_stepped = True
        self._bucket_capture_open = False
        Fn.bump_weight_generation()

    def on_graph_replay(self):
        """A captured step was replayed: its kernels advanced the device step counters; advance the
        host mirrors and every stepped parameter's ``state["step"]`` to match."""
        for key in self._captured or ():
            ds = self._dsteps.get(key)
            if ds is None:
                continue
            ds[1] += 1
            for p in ds[2]:
                self.state[p]["step"] += 1

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dsteps.clear()  # re-seeded from the loaded host step counts at the next step

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._reducer_stepped:
            self._reducer_stepped = False
            return loss
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if capturing:
            self._captured = []
        self._step_subset(None)
        Fn.bump_weight_generation()
        return loss

    @torch.no_grad()
    def step_params(self, params):
        """Update only ``params`` (one bucket of the bucket engine); see FusedSGD.step_params."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing() and not self._bucket_capture_open:
            self._captured = []  # the first bucket of a captured backward: this capture's launch keys
            self._bucket_capture_open = True
        gid = FusedSGD._group_index(self)
        by_group = {}
        for p in params:
            gi = gid.get(id(p))
            if gi is not None and p.grad is not None:
                by_group.setdefault(gi, []).append(p)
        for gi in sorted(by_group):
            self._step_group(gi, self.param_groups[gi], by_group[gi])

    def _step_subset(self, ids):
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None and (ids is None or id(p) in ids)]
            if params:
                self._step_group(gi, group, params)

    def _step_group(self, gi, group, params):
        for p in params:
            st = self.state[p]
            if "step" not in st:
                st["step"] = 0
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["step"] += 1
        # bias correction is per parameter (torch.optim.Adam): one launch per distinct step count
        by_step = {}
        for p in params:
            by_step.setdefault(self.state[p]["step"], []).append(p)
        for step, sub in sorted(by_step.items()):
            self._update(gi, group, sub, step)

    def _update(self, gi, group, params, step):
        b1, b2 = group["betas"]
        if params[0].is_cuda:
            entries = []
            for p in params:
                st = self.state[p]
                entries.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                st["exp_avg_sq"].data_ptr(), 0, p.numel()))
            key = (gi, len(params), params[0].data_ptr())
            table, chunks = self._tables.setdefault(key, _TableCache()).get(entries, params[0].device)
            ds = self._dsteps.get(key)
            if ds is None or ds[1] != step - 1:
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("FusedAdam: step counters must be seeded by an eager step before capture")
                ds = self._dsteps[key] = [torch.full((1,), step - 1, dtype=torch.int32, device=params[0].device),
                                          step - 1, params]
            ds[0].add_(1)  # captured with the step: every replay advances the device count
            ds[1], ds[2] = step, params
            if self._captured is not None and torch.cuda.is_current_stream_capturing():
                self._captured.append(key)
            _ext.hip_ops().mt_adam(table, chunks, group["lr"], b1, b2, group["eps"], group["weight_decay"], step,
                                   group["decoupled"], group["grad_scale"], ds[0])
            return
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        for p in params:
            st = self.state[p]
            g = p.grad * group["grad_scale"]
            if group["weight_decay"]:
                if group["decoupled"]:
                    p.mul_(1 - group["lr"] * group["weight_decay"])
                else:
                    g = g + group["weight_decay"] * p
            st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = st["exp_avg_sq"].sqrt() / math.sqrt(bc2) + group["eps"]
            p.addcdiv_(st["exp_avg"], denom, value=-group["lr"] / bc1)
