#!/usr/bin/env python3
"""Per-(kernel, grid) breakdown of a rocprofv3 kernel-trace database (run_results.db).

Groups dispatches by kernel name, grid (workgroups) and workgroup size and prints calls and time per
step, largest total first -- the view that shows which launches are grid-bound (few workgroups for a
256-CU chip) rather than just which kernel names cost most.

  python3 tools/rocpd_by_grid.py gpurun_out/s44/profsmall_batch_32/run_results.db --steps 105 --top 60
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=105, help="steps in the trace (timed + warmup replays)")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    c = sqlite3.connect(a.db).cursor()
    q = """select s.display_name, d.grid_size_x / d.workgroup_size_x, d.grid_size_y, d.workgroup_size_x,
                  count(*), avg(d.end - d.start) / 1000.0
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by 1, 2, 3, 4"""
    rows = sorted(c.execute(q).fetchall(), key=lambda r: -r[4] * r[5])
    print(f"{'kernel':60s} {'grid':>11s} {'wg':>5s} {'n/step':>7s} {'mean us':>8s} {'us/step':>8s}")
    for name, gx, gy, wg, n, us in rows[:a.top]:
        print(f"{name[:60]:60s} {gx:6d} x {gy:3d} {wg:5d} {n / a.steps:7.1f} {us:8.2f} {n * us / a.steps:8.1f}")
    print(f"total us/step {sum(r[4] * r[5] for r in rows) / a.steps:.1f}")


if __name__ == "__main__":
    main()
