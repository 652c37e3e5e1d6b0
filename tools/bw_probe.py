#!/usr/bin/env python3
"""HBM write / read / copy rates on this GPU for the R50 stage-1 tensor size (the roofline the
write-heavy conv epilogues are judged against):  python tools/bw_probe.py [--gb 1.64]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.ew_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.64)
    a = ap.parse_args()
    rows = int(a.gb * 1e9 / 2 / 1024) // 4 * 4
    x = torch.randn(rows, 1024, device="cuda").bfloat16()
    y = torch.empty_like(x)
    gb = x.numel() * 2 / 1e9
    t = timeit(lambda: y.fill_(1.0), iters=10)
    print(f"write-only fill_ {gb:.2f} GB: {t:8.1f} us  {gb / t * 1e6 / 1e3:6.2f} TB/s", flush=True)
    t = timeit(lambda: y.copy_(x), iters=10)
    print(f"copy {gb:.2f} GB -> {gb:.2f} GB: {t:8.1f} us  {2 * gb / t * 1e6 / 1e3:6.2f} TB/s (read+write)", flush=True)
    t = timeit(lambda: x.sum(dtype=torch.float32), iters=10)
    print(f"read-only sum {gb:.2f} GB: {t:8.1f} us  {gb / t * 1e6 / 1e3:6.2f} TB/s", flush=True)
    s = x[: rows // 4]
    t = timeit(lambda: y.view(4, -1, 1024).copy_(s.unsqueeze(0).expand(4, -1, -1)), iters=10)
    print(f"broadcast-copy {gb / 4:.2f} GB -> {gb:.2f} GB: {t:8.1f} us  {1.25 * gb / t * 1e6 / 1e3:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
