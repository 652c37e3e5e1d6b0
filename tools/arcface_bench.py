#!/usr/bin/env python3
"""ArcFace head step time (forward + backward of ArcMarginProduct + CE on the features and the
class weights), fused (csrc/arcface.hip) vs the unfused kernel path, and the peak extra memory.

    python tools/arcface_bench.py [--batch 1024] [--classes 10000,100000] [--dim 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from ddp_classification_pytorch_amd.ops import functional as Fn  # noqa: E402


def step(x, W, lab):
    x.grad = W.grad = None
    loss, _, _ = Fn.arcface_loss(x, W, lab, 30.0, 0.5, True)
    loss.backward()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--classes", default="10000,100000")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mode", default="both", choices=["both", "fused", "unfused"])
    ap.add_argument("--graph", action="store_true",
                    help="time HIP-graph replays of the head step (as bench.py / main.py run it): no host launch cost")
    a = ap.parse_args()
    _ext.hip_ops()
    dev = torch.device("cuda", 0)
    print(f"{'B':>6s} {'C':>7s} {'D':>4s} | {'fused us':>9s} {'unfused us':>10s} {'speedup':>7s} | "
          f"{'fused MB':>8s} {'unfused MB':>10s}")
    for C in (int(c) for c in a.classes.split(",")):
        torch.manual_seed(0)
        x = torch.randn(a.batch, a.dim, device=dev).requires_grad_(True)
        W = (torch.randn(C, a.dim, device=dev) * 0.05).requires_grad_(True)
        lab = torch.randint(0, C, (a.batch,), device=dev)
        res = {}
        modes = {"both": ("1", "0"), "fused": ("1",), "unfused": ("0",)}[a.mode]
        for fused in modes:
            os.environ["DCP_ARCFACE_FUSED"] = fused
            for _ in range(3):
                step(x, W, lab)
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            step(x, W, lab)
            torch.cuda.synchronize()
            peak = (torch.cuda.max_memory_allocated() - base) / 2**20
            run = lambda: step(x, W, lab)  # noqa: E731
            if a.graph:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    step(x, W, lab)
                torch.cuda.current_stream().wait_stream(side)
                g = torch.cuda.CUDAGraph()
                x.grad = W.grad = None
                with torch.cuda.graph(g):
                    loss, _, _ = Fn.arcface_loss(x, W, lab, 30.0, 0.5, True)
                    loss.backward()
                run = g.replay
                for _ in range(3):
                    run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[fused] = (e0.elapsed_time(e1) / a.iters * 1e3, peak)
        os.environ.pop("DCP_ARCFACE_FUSED", None)
        f, u = res.get("1", (float("nan"), 0.0)), res.get("0", (float("nan"), 0.0))
        print(f"{a.batch:6d} {C:7d} {a.dim:4d} | {f[0]:9.1f} {u[0]:10.1f} {u[0] / f[0]:7.2f} | {f[1]:8.1f} {u[1]:10.1f}",
              flush=True)


if __name__ == "__main__":
    main()
