#!/usr/bin/env python3
"""Dispatch-by-dispatch timeline of ONE training step from a rocprofv3 (rocpd) database:
the dispatches between the last two optimizer-step kernels, with duration, gap to the
previous dispatch, grid, LDS and register counts.

    python tools/step_timeline.py gpurun_out/prof/run_results.db [--marker mt_sgd_kernel]
"""
import argparse
import re
import sqlite3
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="mt_sgd_kernel")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, accum_vgpr_count, "
                     "sgpr_count from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        print("need two marker dispatches", file=sys.stderr)
        return 1
    seg = rows[marks[-2] + 1: marks[-1] + 1]
    t0 = seg[0][1]
    busy = 0.0
    prev_end = rows[marks[-2]][2]
    for name, s, e, gx, wx, lds, vg, ag, sg in seg:
        d = (e - s) / 1e3
        busy += d
        gap = (s - prev_end) / 1e3
        prev_end = e
        if d < a.min_us:
            continue
        nm = re.sub(r"\(.*\)$", "", name)[:60]
        print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} {gap:6.1f}  {nm:60s} wg={gx // max(wx, 1):6d} lds={lds:6d} "
              f"v={vg}/{ag} s={sg}")
    span = (seg[-1][2] - seg[0][1]) / 1e3
    print(f"# {len(seg)} dispatches, busy {busy / 1e3:.2f} ms, span {span / 1e3:.2f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
