#!/bin/bash
# TResNet-M check: its stem/s2d/model tests, two headline-config benches and a kernel profile
set -e
set -o pipefail
O=gpurun_out/${1:-tres}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "s2d or stem or tresnet" > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --config tresnet --steps 20 --warmup 5 > $O/tres_$r.log 2>&1
  grep -o '"value": [0-9.]*' $O/tres_$r.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tres -o run -- python3 -u bench.py --config tresnet --steps 8 --warmup 2 > $O/prof_tres.log 2>&1
echo done
