"""Barrier timestamps of the ping-pong 256 x 256 tap GEMM (timing instrumentation).

    python tools/pp_stamps.py --shape 16 [--batch 1024] [--cfg "tg_big=1"]

Runs one forward conv of an R50 shape (tools/conv_bench.py indices) with g_tune[kAblate] |= 16:
workgroups 0..7 of the 8-wave big tile record, per wave, s_memtime at arrival and release of every
ping-pong barrier (csrc/conv_igemm.hip tap_gemm_big_kernel) and their HW_ID register.  Prints each
wave's SIMD, and per wave group the median cycles of its segments: time from a release to its next
arrival (the wave's own work in that interval) and the wait at the barrier.
"""
from __future__ import annotations

import argparse
import os
import statistics as st
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext, tuning  # noqa: E402
from tools.conv_bench import R50  # noqa: E402

SLOTS = 72


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--cfg", default="tg_big=1")
    a = ap.parse_args()
    K = _ext.hip_ops()
    dev = torch.device("cuda", 0)
    Ci, Co, k, s, H, _ = R50[a.shape]
    p = k // 2
    x = torch.randn(a.batch, H, H, Ci, device=dev).bfloat16()
    w = torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5
    wb, _ = K.weight_prep(w, 0, True)
    buf = torch.zeros(8 * 8 * SLOTS, dtype=torch.long, device=dev)
    tuning.apply(K, a.cfg)
    K.conv_fwd(x, wb, s, p, True)
    K.set_tg_stamps(buf)
    K.set_tuning(tuning.slot("ablate"), 16)
    K.conv_fwd(x, wb, s, p, True)
    torch.cuda.synchronize()
    K.set_tuning(tuning.slot("ablate"), 0)
    K.set_tg_stamps(None)
    tuning.apply(K, "", reset=True)
    b = buf.view(8, 8, SLOTS).cpu()
    print(f"shape {a.shape}: {Ci}->{Co} k{k} s{s} {H}x{H}, batch {a.batch}, cfg {a.cfg}")
    for wg in range(8):
        hw = [int(b[wg, wv, SLOTS - 1]) for wv in range(8)]
        simd = [(h >> 4) & 3 for h in hw]
        cu = [(h >> 8) & 15 for h in hw]
        n = [int((b[wg, wv, :SLOTS - 2] != 0).sum()) for wv in range(8)]
        if min(n) < 8:
            print(f"wg {wg}: no stamps")
            continue
        t0 = min(int(b[wg, wv, 0]) for wv in range(8))
        line = f"wg {wg} simd per wave {simd} cu {cu[0]}"
        for g, waves in ((0, range(0, 4)), (1, range(4, 8))):
            work, wait = {0: [], 1: []}, []
            for wv in waves:
                ev = [int(v) - t0 for v in b[wg, wv, :min(n)]]
                arr, rel = ev[0::2], ev[1::2]
                wait += [r - q for q, r in zip(arr, rel)]
                for i in range(1, len(arr)):
                    work[i % 2].append(arr[i] - rel[i - 1])
            line += (f" | grp {g}: work even/odd {st.median(work[0]):.0f}/{st.median(work[1]):.0f}"
                     f" wait {st.median(wait):.0f}")
        print(line)
        if wg == 0:
            for wv in range(8):
                ev = [int(v) - t0 for v in b[wg, wv, :min(n)]]
                print(f"  wave {wv} simd {simd[wv]}: " + " ".join(f"{e}" for e in ev[:24]))


if __name__ == "__main__":
    main()
