#!/bin/bash
# GPU tests ($1 filter), the forward-conv epilogue / ablation timings and the headline bench.
set -e
O=gpurun_out/fwd; mkdir -p $O
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 400 python -u tools/fwd_epi_bench.py --batch 1024 > $O/fwd_epi.txt 2>&1
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
grep -o '"value": [0-9.]*' $O/bench.log
echo fwd done
