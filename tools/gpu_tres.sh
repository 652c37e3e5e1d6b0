#!/bin/bash
set -e
O=gpurun_out/${1:-tres}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tresnet or dwconv or chan_scale or parity or workloads or dgrad_bn or leaky" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 240 python -u bench.py --config tresnet --steps 20 --warmup 5 > $O/bench_tresnet.log 2>&1; tail -1 $O/bench_tresnet.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --config tresnet --steps 6 --warmup 2 > $O/prof.log 2>&1
echo prof done
