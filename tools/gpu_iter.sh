#!/bin/bash
# One build->measure iteration on the GPU box: kernel numerics tests (-k filter in $1),
# the headline bench, optionally per-shape conv timings ($2 = "conv") and a rocprofv3
# kernel trace ($3 = "prof").  Every GPU step has its own time limit; stops at the first failure.
set -e
O=gpurun_out/iter; mkdir -p $O
K="${1:-}"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
grep -o '"value": [0-9.]*' $O/bench.log
if [ "$2" = "conv" ]; then
  timeout -k 10 300 python -u tools/conv_bench.py --batch 512 --no-miopen > $O/conv_b512.txt 2>&1
  tail -1 $O/conv_b512.txt
fi
if [ "$3" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1
fi
echo iter done
