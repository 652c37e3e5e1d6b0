#!/usr/bin/env python3
"""Counter table of the ``pmc6`` passes (tools/gpu_round.sh): for every (shape, pass) block of
tools/pmc_r6.py, the kernels that ran inside the counted block (tuning dispatches excluded),
averaged per call, with

  us      kernel time per call
  MFMA%   SQ_VALU_MFMA_BUSY_CYCLES / (time x 2.4 GHz x 1024 SIMDs), as profiles/r4
  LDSc%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  ldsI/w  SQ_INSTS_LDS per wave;   wLDS  SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  wAny    SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  L2->L1  TCP_TCC_READ_REQ_sum x 64 B (the L2 -> LDS-DMA / vector-L1 read bytes), GB/s
  L2hit   TCC_HIT / (TCC_HIT + TCC_MISS)
  HBMrd / HBMwr   2 x FETCH_SIZE (upper estimate, tools/pmc_report.py) / WRITE_SIZE, MB and GB/s

    python tools/pmc_r6_report.py gpurun_out/<tag>/pmc6 [--log gpurun_out/<tag>/pmc6_p1.log]
"""
import argparse
import collections
import csv
import glob
import os
import re

CLK = 2.4e9
CUS = 256


def load(path):
    """dispatches in order: (name, seconds, {counter: value})"""
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        did = int(r["Dispatch_Id"])
        e = rows.setdefault(did, [r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, {}])
        e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def blocks(disp):
    """lists of the dispatches between each start (exp) and end (sin) marker"""
    out, cur = [], None
    for name, t, c in disp:
        if re.search(r"exp_kernel", name):
            cur = []
        elif re.search(r"sin_kernel", name):
            if cur is not None:
                out.append(cur)
            cur = None
        elif cur is not None:
            cur.append((name, t, c))
    return out


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("dcp::", "")
    return n.replace("(anonymous namespace)::", "")[:44]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", help="directory holding pass subdirectories p1..pN (run_counter_collection.csv)")
    ap.add_argument("--log", default=None, help="the program's stdout (BLOCK labels)")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    passes = []
    for d in sorted(glob.glob(os.path.join(a.dir, "p*"))):
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if f:
            passes.append(blocks(load(f[0])))
    labels = []
    if a.log and os.path.exists(a.log):
        labels = [ln.split(" ", 1)[1].strip() for ln in open(a.log) if ln.startswith("BLOCK ")]
    nb = min(len(p) for p in passes)
    print(f"{'block':34s} {'kernel':44s} {'us':>7s} {'MFMA%':>6s} {'LDSc%':>6s} {'ldsI/w':>7s} {'wLDS':>5s} "
          f"{'wAny':>5s} {'L2->L1':>7s} {'L2hit':>6s} {'HBMrd':>7s} {'HBMwr':>7s} {'rdGB/s':>7s} {'wrGB/s':>7s}")
    for b in range(nb):
        # per kernel name: merge the counters every pass recorded for that kernel's dispatches
        agg = collections.OrderedDict()
        for p in passes:
            for name, t, c in p[b]:
                e = agg.setdefault(short(name), {"n": collections.Counter(), "t": collections.Counter(), "c": {}})
                pid = id(p)
                e["n"][pid] += 1
                e["t"][pid] += t
                for k, v in c.items():
                    e["c"][k] = e["c"].get(k, 0.0) + v
        lab = labels[b] if b < len(labels) else f"block {b}"
        for kname, e in agg.items():
            ncall = max(e["n"].values())
            npass = len(e["n"])
            t = sum(e["t"].values()) / max(1, sum(e["n"].values()))  # mean per call over passes
            c = {k: v / ncall for k, v in e["c"].items()}  # per call (each counter comes from one pass)
            wc = max(1.0, c.get("SQ_WAVE_CYCLES", 0.0))
            waves = max(1.0, c.get("SQ_WAVES", 0.0))
            mf = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, t * CLK * CUS * 4)
            ldsc = 100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0.0))
            hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
            l2l1 = c.get("TCP_TCC_READ_REQ_sum", 0.0) * 64.0
            rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024.0  # as tools/pmc_report.py: gfx950 counts wide reads at half
            wr = c.get("WRITE_SIZE", 0.0) * 1024.0
            print(f"{lab[:34]:34s} {kname:44s} {t * 1e6:7.1f} {mf:6.1f} {ldsc:6.2f} "
                  f"{c.get('SQ_INSTS_LDS', 0.0) / waves:7.0f} {c.get('SQ_WAIT_INST_LDS', 0.0) / wc:5.2f} "
                  f"{c.get('SQ_WAIT_INST_ANY', 0.0) / wc:5.2f} {l2l1 / max(t, 1e-9) / 1e9:7.0f} "
                  f"{100.0 * hit / max(1.0, hit + miss):6.1f} {rd / 1e6:7.1f} {wr / 1e6:7.1f} "
                  f"{rd / max(t, 1e-9) / 1e9:7.0f} {wr / max(t, 1e-9) / 1e9:7.0f}"
                  + ("" if npass == len(passes) else f"  (in {npass}/{len(passes)} passes)"))


if __name__ == "__main__":
    main()
