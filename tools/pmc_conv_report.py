#!/usr/bin/env python3
"""Per-dispatch table of the ``pmcconv`` PMC passes (tools/gpu_round.sh): every conv kernel
dispatch of tools/pmc_conv.py in program order, with its time, MFMA-busy share, LDS bank-conflict
share, wait / issue shares, L2 hit rate and HBM-side read bytes.

    python tools/pmc_conv_report.py gpurun_out/<tag>
"""
import collections
import csv
import os
import re
import sys

PEAK_HZ = 2.4e9
SIMDS = 256 * 4


def load(d):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        did = int(r["Dispatch_Id"])
        e = rows.setdefault(did, {"name": re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
                                  .replace("dcp::", ""),
                                  "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main():
    d = sys.argv[1]
    p1, p2, p3 = (load(os.path.join(d, f"pmcc{i}")) for i in (1, 2, 3))
    keep = lambda e: re.search(r"tap_gemm|conv3x3|stem", e["name"])
    p1, p2, p3 = [e for e in p1 if keep(e)], [e for e in p2 if keep(e)], [e for e in p3 if keep(e)]
    print(f"{'kernel':58s} {'us':>7s} {'MFMA%':>6s} {'LDSc%':>6s} {'wait':>5s} {'inst':>5s} {'L2hit':>6s} "
          f"{'rdMB':>8s} {'rdGB/s':>7s}")
    for a, b, c in zip(p1, p2, p3):
        wc = max(1.0, a.get("SQ_WAVE_CYCLES", 0.0))
        mf = 100.0 * a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, a["t"] * PEAK_HZ * SIMDS)
        lds = 100.0 * a.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, a.get("SQ_LDS_IDX_ACTIVE", 0.0))
        hit = b.get("TCC_HIT_sum", 0.0)
        miss = b.get("TCC_MISS_sum", 0.0)
        rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024.0
        print(f"{a['name'][:58]:58s} {a['t'] * 1e6:7.1f} {mf:6.1f} {lds:6.2f} {a.get('SQ_WAIT_ANY', 0) / wc:5.2f} "
              f"{a.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} {100 * hit / max(1.0, hit + miss):6.1f} {rd / 1e6:8.1f} "
              f"{rd / max(1e-9, c['t']) / 1e9:7.0f}")


if __name__ == "__main__":
    main()
