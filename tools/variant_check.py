#!/usr/bin/env python3
"""Per-shape check of every autotuner candidate (kTgCfgs) against the heuristic on the conv shapes of
a small-batch ResNet-50 step: forward output (same k order: expected bitwise equal but for stream-K),
forward BN statistics (vs the fp32 statistics of the bf16 output), data gradient.  Finds a
variant-specific defect the whole-model check (tests/test_autotune_variants_gpu.py) can only see
through the running statistics.

    python tools/variant_check.py [--batch 16] [--size 64]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext, tuning  # noqa: E402
from ddp_classification_pytorch_amd.ops import _ref  # noqa: E402
from tests.test_autotune_variants_gpu import TG, TG_SLOTS  # noqa: E402
from tools.conv_bench import R50  # noqa: E402


def relerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=64)
    a = ap.parse_args()
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    scale = a.size / 224.0
    bad = 0
    for idx, (Ci, Co, k, s, H, _) in enumerate(R50):
        if idx == 0:
            continue  # the stem (its own kernel)
        H = max(1, int(round(H * scale)))
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        torch.manual_seed(idx)
        x = torch.randn(a.batch, H, H, Ci, device=dev).bfloat16()
        w = torch.randn(Co, k, k, Ci, device=dev) / math.sqrt(k * k * Ci)
        wb, wt = K.weight_prep(w, 0, True)
        dy = torch.randn(a.batch, Ho, Ho, Co, device=dev).bfloat16()
        res = {}
        for ci, cfg in enumerate(TG):
            tuning.apply(K, "", reset=True)
            for sl, v in zip(TG_SLOTS, cfg):
                K.set_tuning(tuning.slot(sl), int(v))
            y, slabs = K.conv_fwd(x, wb, s, p, True)
            st = K.bn_stats(y, slabs)
            dx = K.conv_dgrad(dy, wt, H, H, s, p)
            torch.cuda.synchronize()
            res[ci] = (y.clone(), st.clone(), dx.clone())
        tuning.apply(K, "", reset=True)
        y0, st0, dx0 = res[0]
        sr = _ref.bn_stats(y0.float().cpu(), None)
        line = []
        for ci in range(len(TG)):
            y, st, dx = res[ci]
            ey = relerr(y, y0)
            em = relerr(st[0, 1], sr[0, 1])
            ev = relerr(st[0, 2], sr[0, 2])
            ed = relerr(dx, dx0)
            flag = ey > 1e-2 or em > 1e-4 or ev > 1e-4 or ed > 1e-2
            bad += flag
            line.append(f"{ci}:{'BAD' if flag else 'ok'}" + (f"(y{ey:.1e} m{em:.1e} v{ev:.1e} d{ed:.1e})" if flag else ""))
        print(f"{idx:2d} {Ci}->{Co} k{k} s{s} {H}->{Ho} M={a.batch * Ho * Ho}: " + " ".join(line), flush=True)
    print(f"variants with a mismatch: {bad}")


if __name__ == "__main__":
    main()
