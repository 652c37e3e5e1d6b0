#!/usr/bin/env python3
"""Forward convs of chosen ResNet-50 shapes under chosen g_tune configurations, a few calls each --
the program a rocprofv3 ``--pmc`` pass wraps to compare kernel variants' counters
(``tools/gpu_round.sh pmcconv``).

    python tools/pmc_conv.py --only 13,16 --cfgs "26=0,26=1" [--batch 1024] [--iters 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from tools.conv_bench import R50, _apply  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True)
    ap.add_argument("--cfgs", required=True)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    for idx in (int(i) for i in a.only.split(",")):
        Ci, Co, k, s, H, _ = R50[idx]
        p = k // 2
        x = torch.randn(a.batch, H, H, Ci, device=dev).bfloat16()
        w = torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5
        wb, _ = K.weight_prep(w, 0, True)
        for cfg in a.cfgs.split(","):
            _apply(K, cfg)
            for _ in range(a.iters):
                K.conv_fwd(x, wb, s, p, True)
            torch.cuda.synchronize()
            print(f"shape {idx} cfg {cfg} done", flush=True)
    _apply(K, "")


if __name__ == "__main__":
    main()
