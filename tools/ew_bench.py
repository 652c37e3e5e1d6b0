#!/usr/bin/env python3
"""Bandwidth of the BN elementwise passes (apply+residual+ReLU forward, backward elementwise)
on the ResNet-50 stage-1 tensor at batch 512, under kernel tuning configs (g_tune slots):
    python tools/ew_bench.py ",9=2048,10=16,11=1"
"""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from ddp_classification_pytorch_amd.tuning import slot as tslot  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    K = _ext.hip_ops()
    cfgs = (sys.argv[1] if len(sys.argv) > 1 else "").split(",")
    shapes = [(512, 56, 56, 256), (512, 28, 28, 512), (512, 56, 56, 64)]
    for shp in shapes:
        C = shp[-1]
        x = torch.randn(*shp, device="cuda").bfloat16()
        r = torch.randn(*shp, device="cuda").bfloat16()
        g = torch.randn(*shp, device="cuda").bfloat16()
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
        mu, iv = torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5
        sums = torch.randn(2, C, device="cuda")
        nb = x.numel() * 2
        for cfg in cfgs:
            for i in range(8, 16):
                K.set_tuning(i, 0)
            for kv in filter(None, cfg.split(";")):
                i, v = kv.split("=")
                K.set_tuning(tslot(i), int(v))
            best = [1e9, 1e9, 1e9]
            for _ in range(3):
                best[0] = min(best[0], timeit(lambda: K.bn_act(x, r, sc, sh, 1, 0.0)))
                best[1] = min(best[1], timeit(lambda: K.bn_act(x, None, sc, sh, 1, 0.0)))
                best[2] = min(best[2], timeit(lambda: K.bn_bwd_elemt(g, x, None, sc, sh, mu, iv, sums, 1e-6, 0, 0.0,
                                                                     False)))
            print(f"{str(shp):22s} cfg={cfg or 'default':16s} act+res {best[0]:7.1f}us {3 * nb / best[0] / 1e6:5.2f}TB/s | "
                  f"act {best[1]:7.1f}us {2 * nb / best[1] / 1e6:5.2f}TB/s | bwd_elemt {best[2]:7.1f}us "
                  f"{3 * nb / best[2] / 1e6:5.2f}TB/s", flush=True)
    for i in range(8, 16):
        K.set_tuning(i, 0)


if __name__ == "__main__":
    main()
