"""Direct 64->64 3x3 forward (conv3x3.hip) vs the implicit GEMM at ResNet-50 layer1 shape:
   python tools/c3_bench.py [--batch 1024] [--tune 19=1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    K = _ext.hip_ops()
    x = torch.randn(a.batch, a.hw, a.hw, 64, device="cuda").abs().bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") / 24).bfloat16()
    flops = 2.0 * a.batch * a.hw * a.hw * 64 * 576
    for name, tune in (("igemm", {18: 1}), ("direct-8w-2buf", {}), ("direct-4w-1buf", {19: 1}),
                       ("direct-4w-2buf", {19: 2})):
        for k, v in tune.items():
            K.set_tuning(k, v)
        for _ in range(3):
            K.conv_fwd(x, w, 1, 1, True)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            K.conv_fwd(x, w, 1, 1, True)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1000 / a.iters
        print(f"{name:12s} {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
        for k in tune:
            K.set_tuning(k, 0)


if __name__ == "__main__":
    main()
