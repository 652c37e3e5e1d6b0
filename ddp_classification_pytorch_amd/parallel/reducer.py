"""Bucketed gradient all-reduce with the optimizer step fused per bucket, graph-capturable.

The reference wraps its model in ``DistributedDataParallel`` and steps the optimizer after the
whole backward (BASELINE/main.py:149,153,280-281; ARCFACE/arc_main.py:238-243,329-330).  torch's
C++ Reducer cannot be captured into a HIP graph, and its optimizer step waits for the last bucket.
:class:`BucketReducer` is this framework's replacement (SURVEY.md §7.1 "optimizer fused per DDP
bucket", §5.8 items 1-3):

* parameters are grouped into buckets in the order their gradients become ready (the hook order
  of the first backward, broadcast from rank 0 so every rank builds the same layout), a small
  first bucket (4 MiB) then ``bucket_cap_mb`` buckets -- sized for xGMI rings, which are per-link
  bound: a few 25 MiB messages keep each link busy while the backward of earlier layers runs;
* a parameter's gradient is packed into its bucket's flat buffer by ONE multi-tensor launch per
  bucket (``mt_copy``, pre-divided by the world size, optionally rounded to bf16 for a half-size
  all-reduce) when the bucket's last gradient arrives (post-accumulate-grad hook), on a
  dedicated communication stream that forks from the compute stream at that point;
* the bucket is all-reduced on that stream (RCCL over xGMI; gloo on the CPU) and, with an
  attached optimizer, the fused SGD / Adam kernel updates that bucket's parameters right behind
  its all-reduce -- layer4's update runs while layer1's gradients are still being computed and
  reduced; ``optimizer.step()`` after backward is then a no-op for that step;
* ``p.grad`` becomes a view into the (reduced) bucket buffer, like DDP's
  ``gradient_as_bucket_view``, so code that reads gradients after backward (CDR's global top-k
  mask, which therefore runs without the fused optimizer) sees the averaged values;
* at the end of backward (an autograd final callback) the compute stream joins the
  communication stream.  Everything is stream-ordered, no host sync: a whole step -- SyncBN
  collectives included -- can be captured into a HIP graph and replayed (engine/graph.py);
* ``telemetry=True`` records HIP events per step: backward end on the compute stream, first
  bucket start and last bucket done on the communication stream -> the exposed communication
  time (last bucket done after the backward ended) that the bench reports per rank.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import _ext

_COMM_STREAMS = {}
CHUNK = 4096
# Where the bucket work (pack, all-reduce, per-bucket optimizer) runs: a side stream overlapping
# the rest of backward when there is communication to hide (world size > 1), the compute stream at
# world size 1 -- the side stream's fork / join edges cost ~0.15 ms per bucket in a replayed HIP
# graph at batch 32 (6.13 ms plain, 6.30 compute stream, 6.85-6.94 side stream with 5 buckets:
# profiles/r4/ddp_stream_ab_b32.txt).  DCP_COMM_STREAM=1 / 0 forces either.
_SIDE_STREAM_ENV = os.environ.get("DCP_COMM_STREAM", "auto")


def _comm_stream(device, world=2):
    side = _SIDE_STREAM_ENV == "1" or (_SIDE_STREAM_ENV != "0" and world > 1)
    if not side:
        return torch.cuda.current_stream(device)
    s = _COMM_STREAMS.get(device)
    if s is None:
        s = _COMM_STREAMS[device] = torch.cuda.Stream(device=device)
    return s


class _Bucket:
    __slots__ = ("index", "params", "offsets", "numels", "grad_buf", "comm_buf", "views", "pending", "launched",
                 "pack_key", "pack_tab", "unpack_tab", "nbytes", "used_off", "ones")

    def __init__(self, index, params, device, comm_dtype, align=16):
        self.index = index
        self.params = params
        self.offsets, self.numels = [], []
        n = 0
        for p in params:
            self.offsets.append(n)
            self.numels.append(p.numel())
            n += (p.numel() + align - 1) // align * align
        # "used" tail: one slot per parameter, packed as 1/world by every rank that produced its
        # gradient (0 otherwise), so after the all-reduce a slot is > 0 iff SOME rank used the
        # parameter -- torch DDP's find_unused bitmap, riding in the same collective
        self.used_off = n
        n += (len(params) + align - 1) // align * align
        self.grad_buf = torch.zeros(n, dtype=torch.float32, device=device)
        self.comm_buf = (self.grad_buf if comm_dtype == torch.float32
                         else torch.zeros(n, dtype=comm_dtype, device=device))
        self.views = [self.grad_buf[o:o + k].view_as(p) for p, o, k in zip(params, self.offsets, self.numels)]
        self.ones = torch.ones(len(params), dtype=torch.float32, device=device)
        self.nbytes = self.used_off * self.comm_buf.element_size()  # the gradients (the used tail aside)
        self.pending = len(params)
        self.launched = False
        self.pack_key = None
        self.pack_tab = None
        self.unpack_tab = None


class BucketReducer:
    def __init__(self, params, process_group=None, bucket_cap_mb: float = 25.0, first_bucket_mb: float = 4.0,
                 comm_dtype=torch.float32, telemetry: bool = False):
        seen, ps = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        if not ps:
            raise ValueError("BucketReducer: no parameters require gradients")
        self.params = ps
        self.device = ps[0].device
        self.cuda = self.device.type == "cuda"
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # a process group of any size all-reduces (world 1 included: a forced single-GPU DDP run
        # then measures the real RCCL launches); no group at all (plain single process) does not
        self.reduce = dist.is_initialized()
        self.cap = int(bucket_cap_mb * 2**20)
        self.first_cap = int(first_bucket_mb * 2**20) if first_bucket_mb else self.cap
        self.comm_dtype = comm_dtype
        self.index = {id(p): i for i, p in enumerate(ps)}
        self.optimizers = []
        self.telemetry = telemetry
        self.records = []           # per-step (bwd_end, first_start, comm_done) events
        self._ev = None
        self._armed = False
        self._order = []            # hook order of the current backward
        self._rebuilt = False
        self._compute = None
        self._next = 0              # the next bucket index to launch this backward
        self._hold = []             # side-stream case: this backward's packed autograd gradients
        self._bucket_opts = {}      # bucket index -> [(optimizer, its params in the bucket)]
        self._warned_unused = False
        self._build(list(reversed(range(len(ps)))))
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in ps]

    # ------------------------------------------------------------------ layout
    def _build(self, order):
        self.buckets, self.bucket_of = [], [0] * len(self.params)
        cur, size = [], 0
        for i in order:
            p = self.params[i]
            cur.append(i)
            size += p.numel() * (2 if self.comm_dtype == torch.bfloat16 else 4)
            if size >= (self.first_cap if not self.buckets else self.cap):
                self._add_bucket(cur)
                cur, size = [], 0
        if cur:
            self._add_bucket(cur)

    def _add_bucket(self, idxs):
        b = _Bucket(len(self.buckets), [self.params[i] for i in idxs], self.device, self.comm_dtype)
        for i in idxs:
            self.bucket_of[i] = b.index
        self.buckets.append(b)

    def bucket_sizes_mb(self):
        return [b.nbytes / 2**20 for b in self.buckets]

    def _rebuild_from_observed(self):
        """After the first backward: buckets in gradient-ready order, rank 0's order on every rank."""
        order = list(dict.fromkeys(self._order))
        seen = set(order)
        order += [i for i in range(len(self.params)) if i not in seen]
        if self.world > 1:
            t = torch.tensor(order, dtype=torch.int64, device=self.device)
            dist.broadcast(t, 0, group=self.group)
            order = t.tolist()
        # the gradients just reduced move to the new views (p.grad must stay valid for step())
        old = [p.grad for p in self.params]
        self._build(order)
        slot = {}
        for b in self.buckets:
            for k, q in enumerate(b.params):
                slot[id(q)] = (b, k)
        for p, g in zip(self.params, old):
            if g is not None:
                b, k = slot[id(p)]
                b.views[k].copy_(g)
                p.grad = b.views[k]
        self._rebuilt = True

    # ------------------------------------------------------------------ optimizer
    def attach_optimizer(self, opt):
        """Run ``opt``'s fused kernel per bucket right after the bucket's all-reduce (its
        ``step()`` after backward then skips once).  The optimizer must be a FusedSGD / FusedAdam
        over (a subset of) these parameters."""
        if not hasattr(opt, "step_params"):
            raise TypeError("attach_optimizer needs a FusedSGD / FusedAdam (step_params)")
        # every trainable parameter of the optimizer must be reduced (and so stepped) here: its
        # step() after backward becomes a no-op, so a parameter outside the wrapped module (an
        # unwrapped head, a margin weight) would silently never be updated
        outside = [p for g in opt.param_groups for p in g["params"] if p.requires_grad and id(p) not in self.index]
        if outside:
            raise ValueError(f"attach_optimizer: {len(outside)} optimizer parameter(s) are not in the wrapped module "
                             f"(shapes {[tuple(p.shape) for p in outside[:4]]}); wrap them too, or give them their "
                             "own optimizer")
        self.optimizers.append(opt)
        self._bucket_opts = {}
        self._opt_params = {}
        for o in self.optimizers:
            for g in o.param_groups:
                for p in g["params"]:
                    self._opt_params[id(p)] = o

    # ------------------------------------------------------------------ hooks
    def _hook(self, p):
        if not self._armed:
            self._armed = True
            self._order = []
            self._compute = torch.cuda.current_stream(self.device) if self.cuda else None
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            if self.telemetry and self.cuda:
                self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        i = self.index[id(p)]
        self._order.append(i)
        b = self.buckets[self.bucket_of[i]]
        b.pending -= 1
        if b.pending == 0 and self._rebuilt_ready():
            # collectives go out in bucket-index order on every rank (one communicator needs the
            # same call sequence everywhere): a bucket that completes early waits for the ones
            # before it -- with buckets built in gradient-ready order that is rarely a delay
            while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
                self._launch(self.buckets[self._next])
                self._next += 1

    def _rebuilt_ready(self):
        # the first backward only records the ready order; its buckets launch together at the end
        return self._rebuilt

    def _pack_tables(self, b, grads, used):
        """Device tables of the bucket's pack launch: every gradient into its slice, and ``used``
        (ones, or a 0/1 vector when this rank lacks some gradient) into the used tail."""
        from ..ops import functional as Fn

        key = tuple(g.data_ptr() for g in grads) + (used.data_ptr(),)
        if key != b.pack_key:
            esz = b.comm_buf.element_size()
            rows = [(b.comm_buf.data_ptr() + o * esz, g.data_ptr(), 0, 0, 0, n)
                    for g, o, n in zip(grads, b.offsets, b.numels)]
            rows.append((b.comm_buf.data_ptr() + b.used_off * esz, used.data_ptr(), 0, 0, 0, len(b.params)))
            if b.pack_tab is None:
                counts = torch.tensor([(n + CHUNK - 1) // CHUNK for n in b.numels + [len(b.params)]],
                                      dtype=torch.int64)
                ent = torch.repeat_interleave(torch.arange(len(b.numels) + 1, dtype=torch.int64), counts)
                first = torch.repeat_interleave(torch.cumsum(counts, 0) - counts, counts)
                ch = torch.stack([ent, torch.arange(ent.numel(), dtype=torch.int64) - first], 1)
                b.unpack_tab = [None, Fn.table_to_device(ch.to(torch.int32), torch.int32, self.device).view(-1, 2)]
                if self.comm_dtype != torch.float32:
                    urows = [(b.grad_buf.data_ptr() + o * 4, b.comm_buf.data_ptr() + o * b.comm_buf.element_size(),
                              0, 0, 0, n) for o, n in zip(b.offsets + [b.used_off], b.numels + [len(b.params)])]
                    b.unpack_tab[0] = Fn.table_to_device(urows, torch.int64, self.device).view(-1, 6)
            b.pack_tab = Fn.table_to_device(rows, torch.int64, self.device).view(-1, 6)
            b.pack_key = key
        return b.pack_tab, b.unpack_tab[1], b.unpack_tab[0]

    def _launch(self, b):
        b.launched = True
        grads = [p.grad for p in b.params]
        present = [g is not None for g in grads]
        if self.cuda:
            comm = _comm_stream(self.device, self.world)
            comm.wait_stream(self._compute)
            with torch.cuda.stream(comm):
                if self._ev is not None and not any(x.launched for x in self.buckets if x is not b):
                    self._ev[1].record(comm)
                self._reduce_cuda(b, grads, comm)
        else:
            self._reduce_cpu(b, grads)
        # A parameter without a gradient on THIS rank (unused in this forward) contributed zeros to
        # the all-reduce.  If ANOTHER rank used it, it gets the reduced view as its gradient, so the
        # replicas apply the same update (torch DDP gives every rank the reduced bucket view too).
        # If NO rank used it (its used slot summed to 0), it keeps grad None on every rank, as torch
        # DDP with find_unused_parameters leaves it: the optimizer then skips it (no weight decay or
        # momentum on a parameter that took no part).  Deciding that reads the used slots on the host
        # -- a sync paid only by a rank that lacks a gradient, never on the all-used fast path.
        unused = set()
        if not all(present):
            if self.cuda and torch.cuda.is_current_stream_capturing():
                # no host read inside a HIP-graph capture: the zero-gradient view stays (every rank
                # alike); a graphed step with unused parameters is not expected
                pass
            else:
                slots = b.comm_buf[b.used_off:b.used_off + len(b.params)].float().cpu()
                unused = {k for k, ok in enumerate(present) if not ok and float(slots[k]) <= 0.0}
            if not self._warned_unused:
                self._warned_unused = True
                import warnings

                warnings.warn("BucketReducer: some parameters received no gradient on this rank; those another "
                              "rank used get the all-reduced bucket view, those no rank used keep grad None",
                              stacklevel=2)
        for k, (p, v) in enumerate(zip(b.params, b.views)):
            p.grad = None if k in unused else v
        self._step_optimizers(b)

    def _reduce_cuda(self, b, grads, comm):
        K = _ext.hip_ops()
        missing = [k for k, g in enumerate(grads) if g is None]
        used = b.ones
        if missing:  # an unused parameter this step: its bucket slice carries zeros, its used slot 0
            used = b.ones.clone()
            for k in missing:
                b.views[k].zero_()
                grads[k] = b.views[k]
                used[k] = 0.0
            self._hold.append([used])  # read by the pack launch (side stream): alive to the join
        pack, chunks, unpack = self._pack_tables(b, grads, used)
        mode = 2 if self.comm_dtype == torch.bfloat16 else 0
        K.mt_copy(pack, chunks, 1.0 / self.world, mode)
        if comm != self._compute:
            # the fresh autograd gradients are read on the side stream: keep them alive until the
            # compute stream has joined it (_finalize) instead of one record_stream per tensor
            self._hold.append(grads)
        if self.reduce:
            dist.all_reduce(b.comm_buf, group=self.group)
        if unpack is not None:
            K.mt_copy(unpack, chunks, 1.0, 1)

    def _reduce_cpu(self, b, grads):
        with torch.no_grad():
            for k, (g, o, n) in enumerate(zip(grads, b.offsets, b.numels)):
                dst = b.comm_buf[o:o + n]
                if g is None:
                    dst.zero_()
                else:
                    dst.copy_(g.reshape(-1).to(torch.float32) / self.world)
                b.comm_buf[b.used_off + k] = 0.0 if g is None else 1.0 / self.world
            if self.reduce:
                dist.all_reduce(b.comm_buf, group=self.group)
            if b.comm_buf is not b.grad_buf:
                b.grad_buf.copy_(b.comm_buf.float())

    def _step_optimizers(self, b):
        if not self.optimizers:
            return
        groups = self._bucket_opts.get(b.index)
        if groups is None or groups[0] is not b:  # per bucket once (layout or optimizers changed)
            by_opt = {}
            for p in b.params:
                o = self._opt_params.get(id(p))
                if o is not None:
                    by_opt.setdefault(id(o), (o, []))[1].append(p)
            groups = self._bucket_opts[b.index] = (b, list(by_opt.values()))
        if not groups[1]:
            return
        by_opt = {id(o): (o, ps) for o, ps in groups[1]}
        if self.cuda:
            with torch.cuda.stream(_comm_stream(self.device, self.world)):
                for o, ps in by_opt.values():
                    o.step_params(ps)
        else:
            for o, ps in by_opt.values():
                o.step_params(ps)

    def _finalize(self):
        if not self._rebuilt:
            self._rebuild_from_observed()
        for b in self.buckets:  # the rest (unused parameters, the first backward) in index order
            if not b.launched:
                self._launch(b)
        if self.cuda:
            comm = _comm_stream(self.device, self.world)
            if self._ev is not None:
                self._ev[0].record(self._compute)
                self._ev[2].record(comm)
                self.records.append(self._ev)
                self._ev = None
            self._compute.wait_stream(comm)
            self._hold = []  # freed on the compute stream, which now follows the side stream's reads
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        self._next = 0
        for o in self.optimizers:
            o.mark_stepped_by_reducer()
        self._armed = False

    # ------------------------------------------------------------------ telemetry
    def telemetry_summary(self, reset=True):
        """Per step, from HIP events (syncs): backward-end -> last-bucket-done (exposed comm, >= 0),
        first-bucket-start -> last-bucket-done (the comm stream's busy span)."""
        if not self.records:
            return None
        torch.cuda.synchronize(self.device)
        exposed, span = [], []
        for bwd_end, first, done in self.records:
            exposed.append(max(0.0, bwd_end.elapsed_time(done)))
            span.append(first.elapsed_time(done))
        if reset:
            self.records = []
        n = len(exposed)
        return {"steps": n, "exposed_comm_ms": round(sum(exposed) / n, 4), "comm_span_ms": round(sum(span) / n, 4),
                "buckets": len(self.buckets), "bucket_mb": [round(v, 2) for v in self.bucket_sizes_mb()]}


class GradSyncDDP(nn.Module):
    """Data-parallel wrapper over :class:`BucketReducer`: parameters and buffers broadcast from rank 0
    at construction (one coalesced broadcast, the reference DDP's C2), then the module's forward;
    gradients are averaged (and, with :meth:`attach_optimizer`, applied) by the bucket engine."""

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb=25.0, first_bucket_mb=4.0,
                 comm_dtype=torch.float32, telemetry=False, broadcast=True):
        super().__init__()
        self.module = module
        self.process_group = process_group
        if broadcast and dist.is_initialized() and dist.get_world_size(process_group) > 1:
            self._broadcast_state()
        self.reducer = BucketReducer(module.parameters(), process_group, bucket_cap_mb, first_bucket_mb, comm_dtype,
                                     telemetry)

    @torch.no_grad()
    def _broadcast_state(self):
        ts = [t for t in list(self.module.parameters()) + list(self.module.buffers()) if t.numel()]
        by = {}
        for t in ts:
            by.setdefault(t.dtype, []).append(t)
        for group in by.values():
            flat = torch.cat([t.reshape(-1) for t in group])
            dist.broadcast(flat, 0, group=self.process_group)
            o = 0
            for t in group:
                t.copy_(flat[o:o + t.numel()].view_as(t))
                o += t.numel()

    def attach_optimizer(self, opt):
        self.reducer.attach_optimizer(opt)
        return opt

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)
