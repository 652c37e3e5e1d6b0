#!/usr/bin/env python3
"""Join the three rocprofv3 PMC passes of `tools/gpu_measure.sh pmc` into one per-kernel table.

    python tools/pmc_report.py gpurun_out/meas [--steps 3] [--top 30]

Pass 1 (SQ + GRBM): MFMA busy share, LDS bank-conflict share, wave-cycle split.
Pass 2 / 3 (TCC): HBM-side read (FETCH_SIZE, kB) / write (WRITE_SIZE, kB) bytes.

Per kernel name (summed over its dispatches in each pass; the passes run the same program):
  ms/step     - kernel time from pass 1 (PMC runs serialise dispatches and run slower)
  MFMA%pk     - SQ_VALU_MFMA_BUSY_CYCLES / (kernel time x 2.4 GHz x 1024 SIMDs): matrix-core
                busy share against the PEAK clock (a lower bound of the at-clock share;
                GRBM_GUI_ACTIVE reads high on short dispatches, so it is not used as the clock)
  LDSconf%    - SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-active cycle)
  wait/inst/activ - SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY shares of SQ_WAVE_CYCLES
  rdGB/s, wrGB/s  - 2 x FETCH_SIZE (gfx950 counts wide streaming reads at half) and WRITE_SIZE
                over the kernel's pass-2 / pass-3 time; 2 x FETCH is an upper estimate for
                kernels whose reads are not wide 16-byte streams
"""
import argparse
import collections
import csv
import os
import re

PEAK_HZ = 2.4e9
SIMDS = 256 * 4


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("dcp::", "")[:48]


def load(d):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    tim = collections.defaultdict(float)
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = short(r["Kernel_Name"])
        ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in seen[k]:
            seen[k].add(r["Dispatch_Id"])
            tim[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return ctr, tim, {k: len(v) for k, v in seen.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3, help="steps the profiled program ran (warmup + timed)")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c1, t1, n1 = load(os.path.join(a.dir, "pmc1"))
    c2, t2, _ = load(os.path.join(a.dir, "pmc2"))
    c3, t3, _ = load(os.path.join(a.dir, "pmc3"))
    tot = sum(t1.values())
    print(f"# PMC-serialised kernel time {tot * 1e3 / a.steps:.2f} ms/step ({a.steps} steps profiled)")
    print(f"{'kernel':48s} {'calls':>5s} {'ms/step':>8s} {'%time':>6s} {'MFMA%pk':>7s} {'LDSconf%':>8s} "
          f"{'wait':>5s} {'inst':>5s} {'activ':>5s} {'rdGB/s':>7s} {'wrGB/s':>7s} {'GB/step':>8s}")
    for k in sorted(t1, key=lambda k: -t1[k])[: a.top]:
        m = c1[k]
        mfma = 100.0 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, t1[k] * PEAK_HZ * SIMDS)
        lds = 100.0 * m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, m.get("SQ_LDS_IDX_ACTIVE", 0.0))
        wc = max(1.0, m.get("SQ_WAVE_CYCLES", 0.0))
        rd = 2.0 * c2[k].get("FETCH_SIZE", 0.0) * 1024.0
        wr = c3[k].get("WRITE_SIZE", 0.0) * 1024.0
        rbw = rd / max(1e-9, t2.get(k, 0.0)) / 1e9
        wbw = wr / max(1e-9, t3.get(k, 0.0)) / 1e9
        print(f"{k:48s} {n1[k] // a.steps:5d} {t1[k] * 1e3 / a.steps:8.3f} {100 * t1[k] / tot:6.2f} {mfma:7.1f} "
              f"{lds:8.2f} {m.get('SQ_WAIT_ANY', 0) / wc:5.2f} {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"{m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} {rbw:7.0f} {wbw:7.0f} {(rd + wr) / 1e9 / a.steps:8.2f}")
    mf = sum(c1[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for k in c1)
    rd = sum(2.0 * c2[k].get("FETCH_SIZE", 0.0) * 1024.0 for k in c2)
    wr = sum(c3[k].get("WRITE_SIZE", 0.0) * 1024.0 for k in c3)
    print(f"# whole step: MFMA busy {100 * mf / max(1.0, tot * PEAK_HZ * SIMDS):.1f}% of peak-clock SIMD cycles; "
          f"HBM-side {rd / 1e9 / a.steps:.1f} GB read (2 x FETCH) + {wr / 1e9 / a.steps:.1f} GB written per step")


if __name__ == "__main__":
    main()
