#!/bin/bash
set -e
O=gpurun_out/sweep2; mkdir -p $O
for b in 1024 1536 2048; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --batch $b > $O/bench_b$b.log 2>&1
  echo "b=$b $(grep -o '"value": [0-9.]*' $O/bench_b$b.log) $(grep -o '"max_mem_gb": [0-9.]*' $O/bench_b$b.log)"
done
