"""Native shard loader throughput on one GPU: synthetic shard of variable-size uint8 records
(ImageNet-like 256-short-side images), RandomResizedCrop(224)+flip, batches of normalised bf16
NHWC (s2d stem layout) delivered to cuda:0.  Prints one JSON line.

    python tools/loader_bench.py --images 2048 --batch 256 --threads 8 --epochs 2
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd.data import ShardSampler  # noqa: E402
from ddp_classification_pytorch_amd.data.shards import ShardLoader, aug_preset, write_shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--prefetch", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--dir", default=tempfile.gettempdir())
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    path = os.path.join(a.dir, f"loader_bench_{os.getpid()}.dcps")

    def gen():
        for i in range(a.images):
            w = int(rng.integers(256, 400))
            yield rng.integers(0, 256, (256, w, 3), dtype=np.uint8), i % 1000

    t0 = time.time()
    write_shard(path, gen())
    pack_s = time.time() - t0
    try:
        aug, size = aug_preset("nested", train=True, size=224)
        sampler = ShardSampler(list(range(a.images)), num_replicas=1, rank=0, shuffle=True)
        ld = ShardLoader(path, a.batch, sampler=sampler, aug=aug, out_size=size, device="cuda", threads=a.threads,
                         prefetch=a.prefetch, s2d=True, drop_last=True)
        ld.set_epoch(0)
        for _ in ld:  # warm-up epoch (page cache, allocator)
            pass
        torch.cuda.synchronize()
        n, t0 = 0, time.time()
        for ep in range(1, a.epochs + 1):
            ld.set_epoch(ep)
            for x, y in ld:
                n += y.numel()
        torch.cuda.synchronize()
        dt = time.time() - t0
        ld.close()
    finally:
        os.remove(path)
    print(json.dumps({"metric": "shard loader images/s to cuda:0 (RRC224+flip, bf16 NHWC s2d)",
                      "value": round(n / dt, 1), "images": a.images, "batch": a.batch, "threads": a.threads,
                      "prefetch": a.prefetch, "pack_s": round(pack_s, 2)}), flush=True)


if __name__ == "__main__":
    main()
