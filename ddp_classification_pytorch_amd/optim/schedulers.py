"""LR schedules used by the reference workloads.

* StepLR(step_size=10, gamma=0.1) per epoch (BASELINE/main.py:154,312; ARCFACE/arc_main.py:255)
  and MultiStepLR(milestones) (CDR/main.py:340, NESTED/train.py:423) are torch's own
  (re-exported here).
* :class:`LinearWarmup` — per-iteration linear ramp (BASELINE/main.py:170-197
  ramps 1e-6 -> lr; NESTED/train.py:292-295 ramps lr*n/warmUpIter).
"""
from __future__ import annotations

from torch.optim.lr_scheduler import MultiStepLR, StepLR  # noqa: F401


class LinearWarmup:
    """Set lr = start + (target - start) * n / iters for n = 1..iters (per-iteration)."""

    def __init__(self, optimizers, iters: int, target_lr: float, start_lr: float = 0.0):
        self.optimizers = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
        self.iters, self.target, self.start = int(iters), float(target_lr), float(start_lr)
        self.n = 0

    def lr_at(self, n: int) -> float:
        if self.iters <= 0:
            return self.target
        f = min(1.0, n / float(self.iters))
        return self.start + (self.target - self.start) * f

    def step(self) -> float:
        self.n += 1
        lr = self.lr_at(self.n)
        for opt in self.optimizers:
            for g in opt.param_groups:
                g["lr"] = lr
        return lr

    @property
    def done(self) -> bool:
        return self.n >= self.iters

    def state_dict(self):
        return {"n": self.n, "iters": self.iters, "target": self.target, "start": self.start}

    def load_state_dict(self, sd):
        self.n, self.iters, self.target, self.start = sd["n"], sd["iters"], sd["target"], sd["start"]
