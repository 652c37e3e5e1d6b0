#!/usr/bin/env python3
"""The production training loop (main.py) against bench.py's stripped step, same model / batch /
input: ``main.py --workload baseline --model resnet50 --data synthetic-device --batchsize B``
(BASELINE/main.py:272-303's loop: metrics every step, periodic log, per-epoch eval skipped by a
large --eval-every) against ``bench.py --batch B`` (same for ``--graph``).

The loop's rate is the median of its logged window rates (``img_per_s`` in metrics.jsonl: wall
time between log points, each ending in a device sync), first window (warm-up, capture) dropped.

    python tools/loop_vs_bench.py --batch 32 [--graph] [--steps 300] [--log-interval 50]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_loop(a, out):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "main.py"), "--workload", "baseline", "--model", "resnet50",
           "--num-classes", "1000", "--hidden", "512", "--data", "synthetic-device", "--batchsize", str(a.batch),
           "--synthetic-train-size", str(a.batch * a.steps), "--synthetic-val-size", str(a.batch),
           "--epochs", "1", "--eval-every", "1000", "--save-every", "1000", "--log-interval", str(a.log_interval),
           "--optimizer", "SGD", "--lr", "0.1", "--no-syncbn", "--out-dir", out, "--dataset", "imagenet"]
    if a.graph:
        cmd.append("--graph")
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL if not a.verbose else None)
    recs = [json.loads(x) for x in open(os.path.join(out, "metrics.jsonl")) if '"train_iter"' in x]
    rates = [r["img_per_s"] for r in recs[1:]] or [r["img_per_s"] for r in recs]
    gpu = [r["gpu_ms_per_step"] for r in recs[1:] if r.get("gpu_ms_per_step")]
    return statistics.median(rates), (statistics.median(gpu) if gpu else None), rates


def run_bench(a):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--batch", str(a.batch), "--steps",
           str(a.bench_steps), "--warmup", "10"]
    cmd.append("--graph" if a.graph else "--eager")  # bench.py defaults to graph replay on one GPU
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    line = [x for x in out.splitlines() if x.startswith("{")][-1]
    return json.loads(line)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--log-interval", type=int, default=50)
    ap.add_argument("--bench-steps", type=int, default=100)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        loop_ips, loop_gpu_ms, rates = run_loop(a, os.path.join(d, "loop"))
    b = run_bench(a)
    res = {"batch": a.batch, "graph": a.graph, "main_py_img_s": round(loop_ips, 1),
           "main_py_window_img_s": [round(r, 1) for r in rates], "main_py_gpu_ms_per_step": loop_gpu_ms,
           "bench_py_img_s": b["value"], "bench_py_ms_per_step": b["ms_per_step"],
           "loop_over_bench": round(loop_ips / b["value"], 4)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
