#!/bin/bash
# autotuner check: its GPU test, HIP-graph batch 32 / 128 (x2) and the headline batch
set -e
set -o pipefail
O=gpurun_out/${1:-tune_check}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "autotune" > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --batch 32 --graph --steps 50 --warmup 5 > $O/g32_$r.log 2>&1
  echo "b32 graph $(grep -o '"value": [0-9.]*' $O/g32_$r.log)"
  timeout -k 10 240 python -u bench.py --batch 128 --graph --steps 30 --warmup 5 > $O/g128_$r.log 2>&1
  echo "b128 graph $(grep -o '"value": [0-9.]*' $O/g128_$r.log)"
done
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b1024.log 2>&1
echo "b1024 $(grep -o '"value": [0-9.]*' $O/b1024.log)"
