#!/usr/bin/env python3
"""Library-GEMM reference (torch.mm -> hipBLASLt/rocBLAS, bf16) for the ResNet-50
1x1 stride-1 convolutions in NHWC GEMM form, next to our tap-GEMM kernels:
fwd  y[M,Co]  = x[M,Ci] W^T,  dgrad dx[M,Ci] = dy[M,Co] W,  wgrad dW[Co,Ci] = dy^T x."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from tools.conv_bench import R50, timeit  # noqa: E402


def main():
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("BATCH", "256"))
    print(f"{'shape':30s} {'blas fwd':>9s} {'dgrad':>8s} {'wgrad':>8s} | {'ours fwd':>9s} {'dgrad':>8s} {'wgrad':>8s}")
    for Ci, Co, k, s, H, cnt in R50:
        if k != 1 or s != 1:
            continue
        M = N * H * H
        x = torch.randn(M, Ci, device=dev).bfloat16()
        w = torch.randn(Co, Ci, device=dev).bfloat16()
        dy = torch.randn(M, Co, device=dev).bfloat16()
        tb = [timeit(lambda: torch.mm(x, w.t()), 10), timeit(lambda: torch.mm(dy, w), 10),
              timeit(lambda: torch.mm(dy.t(), x), 10)]
        x4 = x.view(N, H, H, Ci)
        dy4 = dy.view(N, H, H, Co)
        wf = w.float().view(Co, 1, 1, Ci)
        wb, wt = K.weight_prep(wf, 0, True)
        to = [timeit(lambda: K.conv_fwd(x4, wb, 1, 0, True), 10), timeit(lambda: K.conv_dgrad(dy4, wt, H, H, 1, 0), 10),
              timeit(lambda: K.conv_wgrad(dy4, x4, 1, 1, 1, 0), 10)]
        print(f"{Ci}->{Co} {H}x{H} x{cnt:<14d} {tb[0]:9.1f} {tb[1]:8.1f} {tb[2]:8.1f} | {to[0]:9.1f} {to[1]:8.1f} {to[2]:8.1f}",
              flush=True)


if __name__ == "__main__":
    main()
