#!/bin/bash
# headline per-GPU batch: 1024 vs 1536 vs 2048 (288 GB HBM leaves room), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s51}; mkdir -p $O
for r in 1 2; do
  for b in ${BATCHES:-1024 1536 2048}; do
    timeout -k 10 400 python -u bench.py --batch $b --steps 12 --warmup 4 > $O/b${b}_$r.log 2>&1 || exit 1
    echo "b$b: $(grep -o '"value": [0-9.]*' $O/b${b}_$r.log) $(grep -o '"max_mem_gb": [0-9.]*' $O/b${b}_$r.log)"
  done
done
