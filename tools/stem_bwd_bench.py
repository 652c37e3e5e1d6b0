"""Fused stem backward (stem.hip stem_bwd: max-pool + BN backward + stem weight gradient) at
ResNet-50 224 px, with the kernel's timing ablations (stem_ablate 1: no MFMA phase, 2: no gather):
   python tools/stem_bwd_bench.py [--batch 1024]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext, tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    K = _ext.hip_ops()
    N, H = a.batch, 112
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(N, H // 2, H // 2, 64, device=dev, generator=g).bfloat16()
    idx = torch.randint(0, 9, dy.shape, device=dev, generator=g, dtype=torch.uint8)
    z = torch.randn(N, H, H, 64, device=dev, generator=g).bfloat16()
    x16 = torch.randn(N, H, H, 16, device=dev, generator=g).bfloat16()
    sc, sh, mu, iv = (torch.rand(64, device=dev, generator=g) + 0.5 for _ in range(4))
    slot = tuning.slot("stem_ablate")
    for name, ab in (("full", 0), ("no-mfma", 1), ("no-gather", 2)):
        K.set_tuning(slot, ab)
        for _ in range(3):
            K.stem_bn_pool_bwd(dy, idx, z, x16, sc, sh, mu, iv, 1)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            K.stem_bn_pool_bwd(dy, idx, z, x16, sc, sh, mu, iv, 1)
        e.record()
        torch.cuda.synchronize()
        print(f"stem_bwd b{N} {name:10s} {s.elapsed_time(e) * 1000 / a.iters:8.1f} us", flush=True)
    K.set_tuning(slot, 0)


if __name__ == "__main__":
    main()
