#!/bin/bash
# fused stem backward ablations (DCP_TUNE 17=a): kernel time per variant from a short kernel trace
O=gpurun_out/stemabl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1 2 3; do
  DCP_FUSED_STEM=1 DCP_TUNE="17=$a" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/p$a -o run -- python3 -u bench.py --steps 4 --warmup 1 > $O/p$a.log 2>&1 || { echo "ablate $a failed"; tail -5 $O/p$a.log; exit 1; }
  echo "ablate $a: $(python3 tools/rocpd_summary.py $O/p$a/run_results.db | grep stem_bwd_kernel)"
done
