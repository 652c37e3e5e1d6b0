#!/usr/bin/env python3
"""Summarise a rocprofv3 `--pmc ... --output-format csv` counter file per kernel
dispatch shape: mean counter values and derived ratios (wait / active shares of
SQ_WAVE_CYCLES, LDS bank-conflict share).

    python tools/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [--filter tap_gemm]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("dcp::", "")[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--filter", default="dcp")
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        if a.filter not in r["Kernel_Name"]:
            continue
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key].add((r["Dispatch_Id"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for key, cs in acc.items():
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        d = sorted(x[1] for x in dur[key])
        line = f"{key[0]:40s} grid={key[1]:8d} lds={key[2]:6d} vgpr={key[3]:3d} t={d[len(d) // 2] / 1e3:8.1f}us"
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    line += f" {c[3:]}={m[c] / wc:5.2f}"
        if "SQ_INSTS_LDS" in m and "SQ_LDS_BANK_CONFLICT" in m:
            line += f" ldsconf/inst={m['SQ_LDS_BANK_CONFLICT'] / max(1, m['SQ_INSTS_LDS']):5.2f}"
        for c in sorted(m):
            if c not in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                line += f" {c}={m[c]:.3g}"
        print(line)


if __name__ == "__main__":
    main()
