#!/bin/bash
# SQ counters of the fused stem backward, full kernel and phase-M-only ablation (DCP_TUNE 17=2)
O=gpurun_out/stempmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_SALU"
for a in 0 2; do
  for ps in 1 2; do
    C=$P; [ $ps = 2 ] && C=$P2
    DCP_FUSED_STEM=1 DCP_TUNE="17=$a" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/a${a}p$ps -o run -- python3 -u bench.py --steps 1 --warmup 1 > $O/a${a}p$ps.log 2>&1 || { echo "pmc a=$a pass $ps failed"; tail -5 $O/a${a}p$ps.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, collections, glob, os
for a in (0, 2):
    tot = collections.defaultdict(float); ns = 0
    for ps in (1, 2):
        for f in glob.glob(f"gpurun_out/stempmc/a{a}p{ps}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "stem_bwd_kernel" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"ablate {a}: " + " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items())))
PY
