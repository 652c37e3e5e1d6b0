"""Peer-memory transport for the SyncBN statistics collectives.

SyncBN (the reference's ``convert_sync_batchnorm``, BASELINE/main.py:148, ARCFACE/arc_main.py:239)
puts one small blocking collective per BN layer and direction on the critical path: per ResNet-50
step 49 all-gathers of (n, mean, M2) forward and 49 all-reduces of (sum g, sum g * xhat) backward,
0.5-16 KB each.  Through RCCL each is a collective launch plus protocol round trips (17 us per call
at world size 1 on MI355X, ``bench.py`` ``comm_probe``).  :class:`PeerExchange` replaces them with
ONE single-workgroup kernel per exchange (``csrc/peer.hip``) over "mailboxes": a buffer in every
rank's HBM, mapped into every other rank's address space through HIP IPC once at setup.  The kernel
stores the rank's floats into every mailbox (remote stores over xGMI), raises a flag per mailbox,
polls its own mailbox's flags, and reads the gathered slots back -- no host involvement, so it is
stream-ordered and HIP-graph capturable like the rest of the step.

Selected per process group with :func:`enable` (``convert_sync_batchnorm(..., transport="peer")``,
``DCP_SYNCBN_TRANSPORT=peer``, ``bench.py``'s SyncBN-peer phase); RCCL stays the default.
Collective setup (every rank, same order).  A rank that cannot map a peer's mailbox (peer access
unavailable) makes every rank fall back to RCCL for that group.

Failure semantics: an exchange waits for the other ranks up to a wall-clock deadline
(``DCP_PEER_TIMEOUT_S``, default 300 s -- long enough for a rank-0 checkpoint or a data-loader
stall, as an RCCL collective would simply wait).  A missed
deadline never returns stale data: the kernel sets ``err`` and writes NaN, every later exchange of
that rank fails the same way at once, and :func:`check_all` (the training loop calls it at every
log interval and epoch end, where it synchronises anyway) raises.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import _ext

MAX_FLOATS = 3 * 4096  # the largest SyncBN payload: (n, mean, M2) x (C1 + C2) of a projection pair
# id(group) -> PeerExchange; each entry holds its group (so the id cannot be reused by another group
# while the entry exists) and lookups also compare the group object itself
_EXCHANGES = {}
_DISABLED = {}  # exchanges switched back to RCCL: mailboxes stay mapped for a later enable()


def _timeout_ms() -> int:
    """The exchange deadline: ``DCP_PEER_TIMEOUT_S`` seconds (default 300, the bench's process-group
    timeout; main.py sets it from ``--pg-timeout`` capped at 300 s)."""
    return max(1, int(float(os.environ.get("DCP_PEER_TIMEOUT_S", "300")) * 1000))


class PeerExchange:
    def __init__(self, group, device, max_floats: int = MAX_FLOATS):
        from torch.multiprocessing.reductions import reduce_tensor

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device(device)
        self.slot = (int(max_floats) + 63) // 64 * 64
        # [2 parities][world][slot] data + [world] int32 flags (zero = no exchange yet)
        self.box = torch.zeros(2 * self.world * self.slot + max(64, self.world), dtype=torch.float32,
                               device=self.device)
        self.epoch = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.timeout_ms = _timeout_ms()
        # fault injection (tests): DCP_PEER_DELAY="rank:seconds:n" -- that rank's host sleeps before
        # issuing its n-th exchange, so the other ranks' exchange kernels wait past the deadline
        self.calls, self._delay = 0, None
        inj = os.environ.get("DCP_PEER_DELAY", "")
        if inj:
            r, sec, nth = inj.split(":")
            if int(r) == self.rank:
                self._delay = (float(sec), int(nth))
        K = _ext.hip_ops()
        handles = [None] * self.world
        dist.all_gather_object(handles, reduce_tensor(self.box), group=group)
        ok, self._peers, ptrs = True, [], []
        for r, (fn, args) in enumerate(handles):
            try:
                t = self.box if r == self.rank else fn(*args)
                if t.device != self.device:
                    K.enable_peer_access(t.device.index)
                self._peers.append(t)  # keeps the mapping alive
                ptrs.append(t.data_ptr())
            except Exception:  # noqa: BLE001 - no peer mapping: the group falls back to RCCL
                ok = False
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        self.ok = bool(flag.item())
        self.boxes = torch.tensor(ptrs if self.ok else [0] * self.world, dtype=torch.int64, device=self.device)
        torch.cuda.synchronize(self.device)
        dist.barrier(group=group)  # every rank mapped every mailbox before anyone's first exchange

    def fits(self, t: torch.Tensor) -> bool:
        return self.ok and t.numel() <= self.slot and t.dtype == torch.float32 and t.device == self.device

    def _tick(self):
        self.calls += 1
        if self._delay is not None and self.calls == self._delay[1]:
            import time

            time.sleep(self._delay[0])

    def all_gather_into_tensor(self, out: torch.Tensor, inp: torch.Tensor):
        """``dist.all_gather_into_tensor`` semantics: out = cat over ranks of inp (fp32)."""
        self._tick()
        src = inp.contiguous().view(-1)
        dst = out.view(-1)
        _ext.hip_ops().peer_exchange(src, dst, self.boxes, self.epoch, self.rank, self.world, self.slot, 0, self.err,
                                     self.timeout_ms)
        return out

    def all_reduce(self, t: torch.Tensor):
        """``dist.all_reduce`` (SUM) in place; the sum runs in rank order, identical on every rank."""
        self._tick()
        flat = t.view(-1)
        _ext.hip_ops().peer_exchange(flat, flat, self.boxes, self.epoch, self.rank, self.world, self.slot, 1,
                                     self.err, self.timeout_ms)
        return t

    def check(self):
        """Raise if an exchange gave up waiting for a rank (a host sync; call outside the hot loop).
        Its output and every later exchange's are NaN (the kernel poisons them), so a run must stop."""
        if int(self.err.item()) != 0:
            raise RuntimeError(
                f"SyncBN peer exchange (rank {self.rank} of {self.world}): a rank did not publish its statistics "
                f"within {self.timeout_ms / 1000:.1f} s (DCP_PEER_TIMEOUT_S); the exchange results are NaN and "
                "the run cannot continue")


def _lookup(table, group):
    ex = table.get(id(group))
    return ex if ex is not None and ex.group is group else None


def enable(group, device=None) -> PeerExchange | None:
    """Create (collectively) the peer transport for ``group``; None if a peer cannot be mapped.
    A transport switched off by :func:`disable` is re-enabled with its mailboxes (no setup)."""
    if group is None or not dist.is_initialized():
        return None
    ex = _lookup(_EXCHANGES, group) or _lookup(_DISABLED, group)
    _DISABLED.pop(id(group), None)
    if ex is None:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        ex = PeerExchange(group, dev)
    _EXCHANGES[id(group)] = ex
    return ex if ex.ok else None


def disable(group):
    """Route ``group``'s SyncBN collectives through RCCL again.  The exchange (and its IPC mappings)
    is kept aside, so a later :func:`enable` reuses it without another collective setup."""
    ex = _lookup(_EXCHANGES, group)
    if ex is not None:
        del _EXCHANGES[id(group)]
        _DISABLED[id(group)] = ex


def exchange_for(group) -> PeerExchange | None:
    if not _EXCHANGES or group is None:
        return None
    ex = _lookup(_EXCHANGES, group)
    return ex if ex is not None and ex.ok else None


def check_all():
    """Raise if any enabled exchange timed out (one host sync per exchange; no-op when none is on).
    Called by the training loop at its log interval / epoch end and by bench.py's peer phase."""
    for ex in list(_EXCHANGES.values()):
        if ex.ok:
            ex.check()


def all_gather_into_tensor(out, inp, group):
    ex = exchange_for(group)
    if ex is not None and ex.fits(inp):
        return ex.all_gather_into_tensor(out, inp)
    dist.all_gather_into_tensor(out, inp, group=group)
    return out


def all_reduce(t, group):
    ex = exchange_for(group)
    if ex is not None and ex.fits(t):
        return ex.all_reduce(t)
    dist.all_reduce(t, group=group)
    return t
