#!/usr/bin/env python3
"""Per-shape conv timing: our gfx950 implicit-GEMM kernels vs MIOpen (stock
torch channels_last bf16) on the 23 unique ResNet-50 conv shapes (SURVEY.md
§2.5.1), forward / data-grad / weight-grad.  Prints TFLOP/s per shape and the
per-step totals weighted by each shape's multiplicity in ResNet-50.

    python tools/conv_bench.py [--batch 256] [--iters 20] [--no-miopen]
    python tools/conv_bench.py --grouped [--batch 128]   # ResNeXt-50 32x4d grouped 3x3 convs
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from ddp_classification_pytorch_amd.tuning import slot as tslot  # noqa: E402

# (Ci, Co, k, stride, H_in, count) at 224px
R50 = [
    (8, 64, 7, 2, 224, 1),
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3), (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1),
    (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1), (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]

# ResNeXt-50 32x4d grouped 3x3 convs: (C, stride, H_in, count), groups = 32
RX50_GROUPED = [(128, 1, 56, 3), (256, 2, 56, 1), (256, 1, 28, 3), (512, 2, 28, 1), (512, 1, 14, 5),
                (1024, 2, 14, 1), (1024, 1, 7, 2)]


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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--grouped", action="store_true", help="ResNeXt-50 grouped convs instead of ResNet-50")
    ap.add_argument("--only", default=None, help="comma-separated shape indices to run")
    ap.add_argument("--cfgs", default=None,
                    help="in-process A/B of tuning configs: 'idx=val;idx=val,idx=val,...' (g_tune slots)")
    a = ap.parse_args()
    if a.grouped:
        return grouped(a)
    if a.cfgs:
        return ab(a)
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    N = a.batch
    tot = {"ours": [0, 0, 0], "miopen": [0, 0, 0]}
    rows = []
    print(f"{'shape':34s} {'fwd us':>8s} {'TF':>6s} {'dgrad':>8s} {'TF':>6s} {'wgrad':>8s} {'TF':>6s} | "
          f"{'mi fwd':>8s} {'mi dg':>8s} {'mi wg':>8s} | roofline us f/d/w (eff %)")
    # roofline: minimum HBM bytes (each operand once; a strided 1x1 reads 1/s^2 of its input) at
    # 5.5 TB/s against the MFMA at 2.0 PF/s (bf16 dense at the clock the chip holds under load)
    HBM, MFMA = 5.5e12, 2.0e15
    ideal_tot = [0.0, 0.0, 0.0]
    only = {int(i) for i in a.only.split(",")} if a.only else None
    for idx, (Ci, Co, k, s, H, cnt) in enumerate(R50):
        if only is not None and idx not in only:
            continue
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        flop = 2.0 * N * Ho * Ho * Co * Ci * k * k
        x = torch.randn(N, H, H, Ci, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5)
        wb, wt = K.weight_prep(w, 0, True)
        dy = torch.randn(N, Ho, Ho, Co, device=dev).bfloat16()
        t_f = timeit(lambda: K.conv_fwd(x, wb, s, p, True), a.iters)
        t_d = timeit(lambda: K.conv_dgrad(dy, wt, H, H, s, p), a.iters) if Ci > 8 else 0.0
        t_w = timeit(lambda: K.conv_wgrad(dy, x, k, k, s, p), a.iters)
        mi = [0.0, 0.0, 0.0]
        if not a.no_miopen:
            xc = x.permute(0, 3, 1, 2)  # channels_last NCHW view
            wc = wb.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            dyc = dy.permute(0, 3, 1, 2)
            mi[0] = timeit(lambda: F.conv2d(xc, wc, stride=s, padding=p), a.iters)
            if Ci > 8:
                mi[1] = timeit(lambda: torch.ops.aten.convolution_backward(
                    dyc, xc, wc, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]), a.iters)
            mi[2] = timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xc, wc, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]), a.iters)
        tf = lambda t: flop / t / 1e6 if t > 0 else 0.0  # noqa: E731
        name = f"{Ci}->{Co} k{k} s{s} {H}->{Ho} x{cnt}"
        xin = N * H * H * Ci * 2 / (s * s if k == 1 else 1)
        yout = N * Ho * Ho * Co * 2
        ideal = [max((xin + yout) / HBM, flop / MFMA) * 1e6 for _ in range(3)]
        ideal[1] = max((N * H * H * Ci * 2 + yout) / HBM, flop / MFMA) * 1e6 if Ci > 8 else 0.0
        eff = [100.0 * i / t if t > 0 else 0.0 for i, t in zip(ideal, (t_f, t_d, t_w))]
        for j in range(3):
            ideal_tot[j] += cnt * ideal[j]
        print(f"{name:34s} {t_f:8.1f} {tf(t_f):6.0f} {t_d:8.1f} {tf(t_d):6.0f} {t_w:8.1f} {tf(t_w):6.0f} | "
              f"{mi[0]:8.1f} {mi[1]:8.1f} {mi[2]:8.1f} | {ideal[0]:6.0f} {ideal[1]:6.0f} {ideal[2]:6.0f} "
              f"({eff[0]:3.0f} {eff[1]:3.0f} {eff[2]:3.0f})", flush=True)
        for i, t in enumerate((t_f, t_d, t_w)):
            tot["ours"][i] += cnt * t
        for i, t in enumerate(mi):
            tot["miopen"][i] += cnt * t
        rows.append(dict(shape=name, flop=flop, ours=[t_f, t_d, t_w], miopen=mi, count=cnt))
    print("per-step totals (ms): ours fwd/dgrad/wgrad = " + "/".join(f"{v / 1e3:.2f}" for v in tot["ours"]) +
          f" sum {sum(tot['ours']) / 1e3:.2f}")
    print("                      roofline          = " + "/".join(f"{v / 1e3:.2f}" for v in ideal_tot) +
          f" sum {sum(ideal_tot) / 1e3:.2f}")
    if not a.no_miopen:
        print("                      miopen            = " + "/".join(f"{v / 1e3:.2f}" for v in tot["miopen"]) +
              f" sum {sum(tot['miopen']) / 1e3:.2f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": N, "rows": rows, "totals_us": tot}, f, indent=1)


def _apply(K, cfg):
    for i in range(40):
        K.set_tuning(i, 0)
    for kv in filter(None, cfg.split(";")):
        i, v = kv.split("=")
        K.set_tuning(tslot(i), int(v))


def ab(a):
    """Time every shape under each tuning config in ONE process (interleaved, so the
    clock / box variance between runs does not decide the comparison)."""
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    N = a.batch
    cfgs = a.cfgs.split(",")
    only = {int(i) for i in a.only.split(",")} if a.only else None
    tot = [[0.0] * 3 for _ in cfgs]
    print(f"{'shape':30s} " + " | ".join(f"{c:>22s}" for c in cfgs))
    for idx, (Ci, Co, k, s, H, cnt) in enumerate(R50):
        if only is not None and idx not in only:
            continue
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, Ci, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5)
        wb, wt = K.weight_prep(w, 0, True)
        dy = torch.randn(N, Ho, Ho, Co, device=dev).bfloat16()
        res = [[0.0] * 3 for _ in cfgs]
        for rep in range(3):
            for ci, cfg in enumerate(cfgs):
                _apply(K, cfg)
                t = [timeit(lambda: K.conv_fwd(x, wb, s, p, True), a.iters),
                     timeit(lambda: K.conv_dgrad(dy, wt, H, H, s, p), a.iters) if Ci > 8 else 0.0,
                     timeit(lambda: K.conv_wgrad(dy, x, k, k, s, p), a.iters)]
                for j in range(3):
                    res[ci][j] = t[j] if rep == 0 else min(res[ci][j], t[j])
        for ci in range(len(cfgs)):
            for j in range(3):
                tot[ci][j] += cnt * res[ci][j]
        name = f"{Ci}->{Co} k{k} s{s} {H}->{Ho} x{cnt}"
        print(f"{name:30s} " + " | ".join(f"{r[0]:6.1f} {r[1]:6.1f} {r[2]:6.1f}" for r in res), flush=True)
    _apply(K, "")
    print("per-step totals (ms): " + " | ".join(
        f"{c}: " + "/".join(f"{v / 1e3:.2f}" for v in t) + f" = {sum(t) / 1e3:.2f}" for c, t in zip(cfgs, tot)))


def grouped(a):
    """ResNeXt-50 grouped 3x3 convs as the model runs them (forward with the fused BN statistics,
    data gradient with the fused BN backward, weight gradient); with --cfgs every shape is timed
    under each tuning config in turn (interleaved in one process)."""
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    N, G = a.batch, 32
    cfgs = a.cfgs.split(",") if a.cfgs else [""]
    tot = [[0.0] * 3 for _ in cfgs]
    mtot = [0.0] * 3
    print(f"{'shape':24s} " + " | ".join(f"{(c or 'default')[:22]:>22s}" for c in cfgs) +
          ("" if a.no_miopen else f" | {'miopen fwd/dg/wg':>22s}"))
    for C, s, H, cnt in RX50_GROUPED:
        Ho = (H + 2 - 3) // s + 1
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(C, 3, 3, C // G, device=dev) / (9 * C // G) ** 0.5).bfloat16()
        dy = torch.randn(N, Ho, Ho, C, device=dev).bfloat16()
        co = [torch.rand(C, device=dev) + 0.5 for _ in range(4)]
        res = []
        for ci, c in enumerate(cfgs):
            _apply(K, c)
            t = [timeit(lambda: K.grouped_conv_fwd_stats(x, w, G, s, 1), a.iters),
                 timeit(lambda: K.grouped_conv_dgrad_bn(dy, w, H, H, G, s, 1, x, *co), a.iters),
                 timeit(lambda: K.grouped_conv_wgrad(dy, x, 3, 3, G, s, 1), a.iters)]
            res.append(t)
            for i, v in enumerate(t):
                tot[ci][i] += cnt * v
        _apply(K, "")
        mi = [0.0, 0.0, 0.0]
        if not a.no_miopen:
            xc, dyc = x.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2)
            wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            mi[0] = timeit(lambda: F.conv2d(xc, wc, stride=s, padding=1, groups=G), a.iters)
            mi[1] = timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xc, wc, None, [s, s], [1, 1], [1, 1], False, [0, 0], G, [True, False, False]), a.iters)
            mi[2] = timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xc, wc, None, [s, s], [1, 1], [1, 1], False, [0, 0], G, [False, True, False]), a.iters)
            for i, v in enumerate(mi):
                mtot[i] += cnt * v
        name = f"C{C} s{s} {H}->{Ho} x{cnt}"
        print(f"{name:24s} " + " | ".join(f"{t[0]:6.1f} {t[1]:7.1f} {t[2]:7.1f}" for t in res) +
              ("" if a.no_miopen else f" | {mi[0]:6.1f} {mi[1]:7.1f} {mi[2]:7.1f}"), flush=True)
    for c, t in zip(cfgs, tot):
        print(f"per-step totals (ms) {c or 'default'}: fwd/dgrad/wgrad = " + "/".join(f"{v / 1e3:.2f}" for v in t) +
              f" sum {sum(t) / 1e3:.2f}")
    if not a.no_miopen:
        print("per-step totals (ms) miopen: " + "/".join(f"{v / 1e3:.2f}" for v in mtot) + f" sum {sum(mtot) / 1e3:.2f}")


if __name__ == "__main__":
    main()
