#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite (rocpd) database.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db --steps 11 [--csv out.csv]

Groups dispatches by kernel name, prints calls, total / mean time, share of
the GPU-busy time and the per-training-step time (total / --steps, the
number of steps the profiled program ran including warm-up), plus the
busy-time and wall span of the whole trace.
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    """Kernel name without its parameter list (the LAST balanced parenthesis group, so names with
    '(anonymous namespace)' keep their kernel part) and without the anonymous-namespace marker."""
    if name.startswith("void at::"):
        name = name.split("(")[0]
    elif name.endswith(")"):
        depth = 0
        for i in range(len(name) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(name[i], 0)
            if depth == 0:
                name = name[:i]
                break
    return name.replace("(anonymous namespace)::", "")[:110]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last-steps", type=int, default=0,
                    help="count only the dispatches of the last K complete steps (each ending with a --marker "
                         "dispatch): warm-up and autotuning dispatches excluded, per step = total / K")
    ap.add_argument("--marker", default="mt_sgd_kernel")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if a.last_steps > 0:
        marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
        if len(marks) < a.last_steps + 1:
            print(f"need {a.last_steps + 1} marker dispatches, found {len(marks)}", file=sys.stderr)
            return 1
        rows = rows[marks[-a.last_steps - 1] + 1: marks[-1] + 1]
        a.steps = a.last_steps
    if not rows:
        print("no kernel dispatches", file=sys.stderr)
        return 1
    agg = {}
    for name, s, e in rows:
        k = short(name)
        d = agg.setdefault(k, [0, 0.0, 1e30, 0.0])
        dur = (e - s) / 1e3
        d[0] += 1
        d[1] += dur
        d[2] = min(d[2], dur)
        d[3] = max(d[3], dur)
    busy = sum(v[1] for v in agg.values())
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) / 1e3
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    hdr = ["kernel", "calls", "total_us", "mean_us", "min_us", "max_us", "pct_busy", "us_per_step"]
    table = [[k, v[0], round(v[1], 1), round(v[1] / v[0], 2), round(v[2], 2), round(v[3], 2),
              round(100 * v[1] / busy, 2), round(v[1] / a.steps, 1)] for k, v in out]
    print(f"# dispatches={len(rows)} gpu_busy_ms={busy / 1e3:.2f} trace_span_ms={span / 1e3:.2f} "
          f"steps={a.steps} busy_ms_per_step={busy / 1e3 / a.steps:.2f}")
    print("%-90s %6s %11s %9s %6s %9s" % ("kernel", "calls", "total_us", "mean_us", "%busy", "us/step"))
    for r in table[: a.top]:
        print("%-90s %6d %11.1f %9.2f %6.2f %9.1f" % (r[0][:90], r[1], r[2], r[3], r[6], r[7]))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(table)
    return 0


if __name__ == "__main__":
    sys.exit(main())
