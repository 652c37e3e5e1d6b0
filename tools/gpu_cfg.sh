#!/bin/bash
# kernel tests ($1 filter) + bench of one config ($2) + its rocprof kernel trace
set -e
O=gpurun_out/cfg_$2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u bench.py --config $2 --steps 20 --warmup 5 > $O/bench.log 2>&1
grep -o '"value": [0-9.]*' $O/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --config $2 --steps 10 --warmup 2 > $O/prof.log 2>&1
echo cfg done
