#!/bin/bash
# HIP-graph step capture: GPU test + eager vs graphed bench at small per-GPU batches.
set -e
O=gpurun_out/${1:-graph}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for b in 16 64 256; do
  for g in "" "--graph"; do
    timeout -k 10 180 python -u bench.py --batch $b --steps 30 --warmup 5 $g > $O/bench_b${b}${g}.log 2>&1 || { tail -20 $O/bench_b${b}${g}.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/bench_b${b}${g}.log').read().strip().splitlines()[-1]); print('b$b', '$g', d['value'], d['ms_per_step'])"
  done
done
