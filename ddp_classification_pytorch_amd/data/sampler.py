"""Rank-sharded sampler with torch DistributedSampler semantics.

Reference: ``DistributedSampler(train/val dataset)`` (BASELINE/main.py:127-128,
ARCFACE/arc_main.py:212-213) — shuffle with ``seed + epoch``; when
``drop_last=False`` the index list is padded by repeating its head so every
rank gets ``ceil(n / world)`` samples; rank r takes ``indices[r::world]``.
``set_epoch`` reshuffles (the reference forgets it in ARCFACE; the engine
here always calls it).  ``sequential_shard=True`` gives contiguous shards.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


class ShardSampler(torch.utils.data.Sampler):
    def __init__(self, dataset, num_replicas=None, rank=None, shuffle=True, seed=0, drop_last=False,
                 sequential_shard=False):
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        if not 0 <= rank < num_replicas:
            raise ValueError(f"rank {rank} outside [0, {num_replicas})")
        self.n = len(dataset)
        self.world, self.rank = num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.sequential_shard = sequential_shard
        self.epoch = 0
        if drop_last and self.n % self.world != 0:
            self.num_samples = math.ceil((self.n - self.world) / self.world)
        else:
            self.num_samples = math.ceil(self.n / self.world)
        self.total_size = self.num_samples * self.world

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def indices(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        assert len(idx) == self.total_size
        if self.sequential_shard:
            return idx[self.rank * self.num_samples:(self.rank + 1) * self.num_samples]
        return idx[self.rank:self.total_size:self.world]

    def __iter__(self):
        return iter(self.indices())

    def __len__(self):
        return self.num_samples

    def state_dict(self):
        return {"epoch": self.epoch, "seed": self.seed}

    def load_state_dict(self, sd):
        self.epoch, self.seed = sd["epoch"], sd["seed"]
