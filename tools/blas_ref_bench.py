#!/usr/bin/env python3
"""Library-GEMM reference points for the ResNet-50 1x1 stride-1 convolutions.

A 1x1 stride-1 NHWC convolution is a plain GEMM ([M, Ci] x [Ci, Co], M = N*H*W), so
torch.mm (hipBLASLt on ROCm) on the same shapes bounds what a well-tuned library tile
reaches on them -- the yardstick for the implicit-GEMM kernels' fwd / dgrad / wgrad times
(tools/conv_bench.py prints those).  Plain GEMM only: no BN statistics, no fused epilogue.

    python tools/blas_ref_bench.py [--batch 1024] [--iters 10]
"""
import argparse

import torch

# (Ci, Co, H, count): the R50 1x1 stride-1 shapes (tools/conv_bench.py R50 list)
SHAPES = [(64, 64, 56, 1), (64, 256, 56, 4), (256, 64, 56, 2), (256, 128, 56, 1), (128, 512, 28, 4),
          (512, 128, 28, 3), (512, 256, 28, 1), (256, 1024, 14, 6), (1024, 256, 14, 5), (1024, 512, 14, 1),
          (512, 2048, 7, 3), (2048, 512, 7, 2)]


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    print(f"{'shape':26s} {'fwd us':>8s} {'TF':>6s} {'dgrad':>8s} {'TF':>6s} {'wgrad':>8s} {'TF':>6s}")
    tot = [0.0, 0.0, 0.0]
    for Ci, Co, H, cnt in SHAPES:
        M = a.batch * H * H
        x = torch.randn(M, Ci, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Ci, Co, device=dev, dtype=torch.bfloat16)
        g = torch.randn(M, Co, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * Ci * Co
        tf = timeit(lambda: torch.mm(x, w), a.iters)
        td = timeit(lambda: torch.mm(g, w.t()), a.iters)
        tw = timeit(lambda: torch.mm(x.t(), g), a.iters)
        for i, t in enumerate((tf, td, tw)):
            tot[i] += t * cnt
        print(f"{Ci:5d}->{Co:<5d} {H:3d}x{H:<3d} x{cnt}    {tf:8.1f} {fl / tf / 1e6:6.0f} {td:8.1f} {fl / td / 1e6:6.0f} "
              f"{tw:8.1f} {fl / tw / 1e6:6.0f}", flush=True)
        del x, w, g
    print(f"per-step totals over these shapes (ms): fwd/dgrad/wgrad = "
          f"{tot[0] / 1e3:.2f}/{tot[1] / 1e3:.2f}/{tot[2] / 1e3:.2f} sum {sum(tot) / 1e3:.2f}")


if __name__ == "__main__":
    main()
