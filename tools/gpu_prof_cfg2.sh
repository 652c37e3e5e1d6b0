#!/bin/bash
# rocprofv3 kernel trace of one bench config: bash tools/gpu_prof_cfg2.sh <tag> <config>
set -e
T=${1:-pc}; C=${2:-tresnet}; O=gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --config $C --steps 6 --warmup 2 > $O/prof.log 2>&1
tail -1 $O/prof.log
