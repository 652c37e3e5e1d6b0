#!/usr/bin/env python3
"""3x3 weight-gradient timing on the ResNet-50 stride-1 shapes: the direct kernel (wgrad3x3.hip)
with its loads or MFMAs ablated (g_tune[2] = 1 / 2), and the implicit-GEMM path (g_tune[15] = 1).
    python tools/wgrad_bench.py [--batch 1024]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from tools.ew_bench import timeit  # noqa: E402

SHAPES = [(56, 64, 64), (28, 128, 128), (14, 256, 256), (7, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    K = _ext.hip_ops()
    N = a.batch
    for H, C, Co in SHAPES:
        dy = torch.randn(N, H, H, Co, device="cuda").bfloat16()
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        flops = 2.0 * N * H * H * Co * 9 * C
        row = {}
        for name, cfg in (("direct", ()), ("noload", ((2, 1),)), ("nomfma", ((2, 2),)), ("forced", ((15, 2),)),
                          ("gemm", ((15, 1),))):
            for i, v in cfg:
                K.set_tuning(i, v)
            row[name] = timeit(lambda: K.conv_wgrad(dy, x, 3, 3, 1, 1), iters=10)
            for i, _ in cfg:
                K.set_tuning(i, 0)
        print(f"H={H:3d} {C:4d}->{Co:4d}: " + " ".join(f"{k} {v:7.1f}us" for k, v in row.items()) +
              f" | direct {flops / row['direct'] / 1e6:5.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
