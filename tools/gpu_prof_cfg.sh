#!/bin/bash
# rocprofv3 kernel trace of one BASELINE config: bash tools/gpu_prof_cfg.sh <config>
set -e
O=gpurun_out/prof_$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 -u bench.py --config $1 --steps 10 --warmup 2 > $O/prof.log 2>&1
echo prof done
