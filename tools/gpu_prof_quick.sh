#!/bin/bash
# quick rocprofv3 kernel trace of the headline step (+ optional DCP_TUNE A/B), summary written on CPU later
set -e
T=${1:-pq}; O=gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1
tail -1 $O/prof.log
if [ -n "$2" ]; then
  DCP_TUNE="$2" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profB -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/profB.log 2>&1
  tail -1 $O/profB.log
fi
