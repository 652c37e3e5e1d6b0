"""Host -> device input pipeline.

Reference: ``DataLoader(num_workers=4, pin_memory=True)`` + ``inputs.cuda(non_blocking=True)``
with ToTensor/Normalize on the CPU workers (BASELINE/main.py:127-131,273-274).

Here:
* workers decode + augment to uint8 HWC and :func:`collate_uint8` stacks them
  (a uint8 batch is 4x smaller than fp32 CHW on the PCIe link);
* :class:`DevicePrefetcher` keeps the next batch in flight on a dedicated HIP
  stream (pinned H2D copy + the ``to_nhwc`` normalisation kernel producing bf16
  NHWC activations with channels padded to 8) while the compute stream runs
  the current step; the compute stream waits on an event, never on the host;
* :class:`SyntheticLoader` serves on-device random uint8 batches (benchmarks,
  BASELINE.json "synthetic" configs) with the same interface.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import functional as Fn
from .transforms import IMAGENET_MEAN, IMAGENET_STD


def collate_uint8(batch):
    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))  # [B,H,W,3] uint8
    labels = torch.tensor([int(b[1]) for b in batch], dtype=torch.int64)
    if len(batch[0]) > 2:
        idx = torch.tensor([int(b[2]) for b in batch], dtype=torch.int64)
        return imgs, labels, idx
    return imgs, labels


def build_loader(dataset, batch_size, sampler=None, shuffle=False, workers=4, drop_last=False, pin_memory=True,
                 worker_init_fn=None, prefetch_factor=4):
    kw = dict(batch_size=batch_size, sampler=sampler, shuffle=shuffle if sampler is None else False,
              num_workers=workers, drop_last=drop_last, pin_memory=pin_memory and torch.cuda.is_available(),
              collate_fn=collate_uint8, worker_init_fn=worker_init_fn)
    if workers > 0:
        kw.update(persistent_workers=True, prefetch_factor=prefetch_factor)
    return torch.utils.data.DataLoader(dataset, **kw)


class DevicePrefetcher:
    """Wraps a loader of (uint8 HWC images, labels[, index]) and yields
    (NHWC activations, labels[, index]) on ``device``."""

    def __init__(self, loader, device, mean=IMAGENET_MEAN, std=IMAGENET_STD, cpad=8, s2d=False):
        self.loader, self.device, self.cpad, self.s2d = loader, torch.device(device), cpad, s2d
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.std = torch.tensor(std, dtype=torch.float32, device=self.device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None

    def __len__(self):
        return len(self.loader)

    @property
    def sampler(self):
        return getattr(self.loader, "sampler", None)

    def _convert(self, batch):
        imgs, labels = batch[0], batch[1]
        imgs = imgs.to(self.device, non_blocking=True)
        labels = labels.to(self.device, non_blocking=True)
        x = Fn.to_device_nhwc(imgs, self.mean, self.std, cpad=self.cpad, nchw=False, in_scale=1.0 / 255.0,
                              s2d=Fn.s2d_for(self.s2d, imgs.shape[1], imgs.shape[2]))
        rest = tuple(b.to(self.device, non_blocking=True) for b in batch[2:])
        return (x, labels) + rest

    def __iter__(self):
        it = iter(self.loader)
        if not self.cuda:
            for b in it:
                yield self._convert(b)
            return
        nxt = None
        try:
            with torch.cuda.stream(self.stream):
                nxt = self._convert(next(it))
        except StopIteration:
            return
        while nxt is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            cur = nxt
            for t in cur:
                t.record_stream(torch.cuda.current_stream(self.device))
            try:
                with torch.cuda.stream(self.stream):
                    nxt = self._convert(next(it))
            except StopIteration:
                nxt = None
            yield cur


class SyntheticLoader:
    """``steps`` batches of on-device random uint8 images (cycling over ``pool`` distinct batches)."""

    def __init__(self, batch_size, steps, size=224, num_classes=1000, device="cuda", pool=2, seed=0,
                 mean=IMAGENET_MEAN, std=IMAGENET_STD, cpad=8, return_index=False, s2d=False):
        self.device = torch.device(device)
        self.steps, self.cpad, self.return_index, self.batch_size = steps, cpad, return_index, batch_size
        self.s2d = Fn.s2d_for(s2d, size, size)
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        self.imgs = [torch.randint(0, 256, (batch_size, size, size, 3), dtype=torch.uint8, generator=g).to(self.device)
                     for _ in range(pool)]
        self.labels = [torch.randint(0, num_classes, (batch_size,), generator=g).to(self.device) for _ in range(pool)]
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.std = torch.tensor(std, dtype=torch.float32, device=self.device)
        self.sampler = None

    def __len__(self):
        return self.steps

    def __iter__(self):
        for i in range(self.steps):
            k = i % len(self.imgs)
            x = Fn.to_device_nhwc(self.imgs[k], self.mean, self.std, cpad=self.cpad, nchw=False, in_scale=1 / 255.0,
                                  s2d=self.s2d)
            if self.return_index:
                idx = torch.arange(k * self.batch_size, (k + 1) * self.batch_size, device=self.device)
                yield x, self.labels[k], idx
            else:
                yield x, self.labels[k]
