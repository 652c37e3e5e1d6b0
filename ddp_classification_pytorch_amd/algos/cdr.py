"""CDR — critical-parameter gradient masking for noisy-label training.

Reference: CDR/main.py:179-215 (`train_one_step`), :218-253 (`train`).
After backward, over all 2-D and 4-D parameters (conv and linear weights):

    metric = |g * w| ;  thr = k-th largest metric, k = int(nonzero_ratio * N)
    g <- g * (|g * w| >= thr) * clip

The reference concatenates the 25.6M-element metric and runs a full
``torch.topk`` every step.  Here (GPU) the threshold comes from a 4-pass 8-bit
radix select over the float bit patterns (``cdr_threshold``) and the mask is
applied in place (``cdr_mask``), both as multi-tensor kernels: nothing is
concatenated or sorted.  CPU uses the reference math.
"""
from __future__ import annotations

from typing import Iterable

import numpy as np
import torch

from .. import _ext

CHUNK = 4096


def _selected(params: Iterable[torch.Tensor]):
    return [p for p in params if p.grad is not None and p.dim() in (2, 4)]


def _table(ps, device):
    entries, chunks = [], []
    for i, p in enumerate(ps):
        if not (p.is_contiguous() and p.grad.is_contiguous() and p.dtype == torch.float32):
            raise RuntimeError("CDR kernels need contiguous fp32 params/grads")
        entries.append((p.data_ptr(), p.grad.data_ptr(), 0, 0, 0, p.numel()))
        chunks.extend((i, c) for c in range((p.numel() + CHUNK - 1) // CHUNK))
    tab = torch.tensor(entries, dtype=torch.int64).view(-1, 6).to(device, non_blocking=True)
    ch = torch.tensor(chunks, dtype=torch.int32).view(-1, 2).to(device, non_blocking=True)
    return tab, ch


@torch.no_grad()
def cdr_mask_gradients(params: Iterable[torch.Tensor], nonzero_ratio: float, clip: float) -> torch.Tensor:
    """Mask gradients in place; returns the threshold (0-dim tensor on the params' device)."""
    ps = _selected(params)
    if not ps:
        return torch.tensor(0.0)
    n = sum(p.numel() for p in ps)
    nz = int(nonzero_ratio * n)
    dev = ps[0].device
    if nz <= 0:
        for p in ps:
            p.grad.zero_()
        return torch.tensor(float("inf"), device=dev)
    if ps[0].is_cuda:
        K = _ext.hip_ops()
        tab, ch = _table(ps, dev)
        state = torch.tensor([0, 0, nz, 0], dtype=torch.int32).to(dev, non_blocking=True)
        thr = K.cdr_threshold(tab, ch, state)
        K.cdr_mask(tab, ch, state, float(clip))
        return thr.reshape(())
    metric = torch.cat([(p.grad * p).abs().view(-1) for p in ps])
    thr = torch.topk(metric, nz)[0][-1]
    for p in ps:
        mask = ((p * p.grad).abs() >= thr).to(p.grad.dtype) * clip
        p.grad.mul_(mask)
    return thr


def clip_schedule(noise_rate: float, num_gradual: int, epoch: int) -> float:
    """CDR/main.py:222-227.  The reference computes a gradual schedule and then
    overrides it with the constant ``1 - noise_rate`` (kept for parity)."""
    sched = np.linspace(1 - noise_rate, 1, num=num_gradual)[::-1]
    _ = sched[epoch] if epoch < num_gradual else None
    return 1.0 - noise_rate
