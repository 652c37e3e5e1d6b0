#!/usr/bin/env python3
"""Forward conv timing on the ResNet-50 shapes: plain store (EPI 0) vs store + BN statistics
(EPI 1), each also with the k-loop loads or the MFMAs ablated (tuning knob 2), and the stem
kernel; prints us and the HBM-side GB/s of the compulsory traffic (input + weight + output).
    python tools/fwd_epi_bench.py [--batch 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from ddp_classification_pytorch_amd.tuning import slot as tslot  # noqa: E402
from tools.ew_bench import timeit  # noqa: E402

# (H, Ci, Co, k, stride)
SHAPES = [(56, 64, 256, 1, 1), (56, 256, 64, 1, 1), (56, 64, 64, 3, 1), (28, 128, 512, 1, 1),
          (28, 512, 128, 1, 1), (28, 128, 128, 3, 1), (14, 256, 1024, 1, 1), (14, 256, 256, 3, 1),
          (7, 512, 512, 3, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    K = _ext.hip_ops()
    N = a.batch
    for H, Ci, Co, k, s in SHAPES:
        x = torch.randn(N, H, H, Ci, device="cuda").bfloat16()
        w = (torch.randn(Co, k, k, Ci, device="cuda") / (k * k * Ci) ** 0.5).bfloat16()
        Ho = (H + 2 * (k // 2) - k) // s + 1
        gb = (x.numel() + w.numel() + N * Ho * Ho * Co) * 2 / 1e9
        flops = 2.0 * N * Ho * Ho * Co * k * k * Ci
        row = []
        for stats in (False, True):
            for abl in (0, 1, 2, 3):
                K.set_tuning(tslot("ablate"), abl)
                us = timeit(lambda: K.conv_fwd(x, w, s, k // 2, stats), iters=10)
                row.append(us)
            K.set_tuning(tslot("ablate"), 0)
        K.set_tuning(tslot("tg_kdepth"), 64)  # 64-deep k-tiles for every shape (disables the 1x1 BK32 heuristic)
        bk64 = timeit(lambda: K.conv_fwd(x, w, s, k // 2, True), iters=10)
        K.set_tuning(tslot("tg_kdepth"), 0)
        print(f"H={H:3d} {Ci:4d}->{Co:4d} k{k}: plain {row[0]:7.1f}us ({gb / row[0] * 1e3:5.2f} TB/s "
              f"{flops / row[0] / 1e6:6.0f} TF/s) noload {row[1]:7.1f} nomfma {row[2]:7.1f} epi-only {row[3]:7.1f} | "
              f"stats {row[4]:7.1f}us ({gb / row[4] * 1e3:5.2f} TB/s) noload {row[5]:7.1f} nomfma {row[6]:7.1f} "
              f"epi-only {row[7]:7.1f} | stats bk64 {bk64:7.1f}", flush=True)
        del x, w
    x = torch.randn(N, 112, 112, 16, device="cuda").bfloat16()
    w = (torch.randn(64, 4, 4, 16, device="cuda") / 16).bfloat16()
    gb = (x.numel() + N * 112 * 112 * 64) * 2 / 1e9
    for stats in (False, True):
        us = timeit(lambda: K.stem_fwd(x, w, stats), iters=10)
        print(f"stem stats={stats}: {us:7.1f}us ({gb / us * 1e3:5.2f} TB/s)", flush=True)
    us = timeit(lambda: K.conv_fwd_geo(x, w, 1, 2, 112, 112, True), iters=10)
    print(f"stem via implicit GEMM: {us:7.1f}us", flush=True)


if __name__ == "__main__":
    main()
