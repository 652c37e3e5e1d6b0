#!/usr/bin/env python3
"""The program a rocprofv3 ``--pmc`` pass wraps to read hardware counters of the conv kernels
the training step ACTUALLY runs: per ResNet-50 shape, forward (BN-statistics epilogue), data
gradient and weight gradient, each called once untimed (the per-shape autotuner settles on
its kernel there, exactly as in ``bench.py``'s warm-up) and then ``--iters`` times.  The
counted blocks are delimited by marker dispatches (an exp / sin over 7 elements) so the report
(``tools/pmc_r6_report.py``) drops the tuning dispatches and keeps only the chosen kernels.

    rocprofv3 --kernel-trace --pmc <counters> -- python3 tools/pmc_r6.py --only 13,16 [--iters 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from tools.conv_bench import R50  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True, help="comma-separated tools/conv_bench.py R50 indices")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--no-autotune", action="store_true", help="the shipped heuristic instead")
    a = ap.parse_args()
    K = _ext.hip_ops()
    from ddp_classification_pytorch_amd.tuning import slot as tslot
    K.set_tuning(tslot("autotune"), 0 if a.no_autotune else 1)
    dev = torch.device("cuda", 0)
    marker = torch.empty(7, device=dev)
    passes = a.passes.split(",")
    for idx in (int(i) for i in a.only.split(",")):
        Ci, Co, k, s, H, _ = R50[idx]
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(a.batch, H, H, Ci, device=dev).bfloat16()
        w = torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5
        wb, wt = K.weight_prep(w, 0, True)
        dy = torch.randn(a.batch, Ho, Ho, Co, device=dev).bfloat16()
        fns = {"fwd": lambda: K.conv_fwd(x, wb, s, p, True),
               "dgrad": lambda: K.conv_dgrad(dy, wt, H, H, s, p),
               "wgrad": lambda: K.conv_wgrad(dy, x, k, k, s, p)}
        for ps in passes:
            if ps == "dgrad" and Ci <= 8:
                continue
            fns[ps]()  # autotuning (if on) happens here, outside the counted block
            torch.cuda.synchronize()
            marker.exp_()  # block start marker
            for _ in range(a.iters):
                fns[ps]()
            torch.cuda.synchronize()
            marker.sin_()  # block end marker
            torch.cuda.synchronize()
            print(f"BLOCK {idx} {Ci}->{Co} k{k} s{s} {H}->{Ho} {ps}", flush=True)


if __name__ == "__main__":
    main()
