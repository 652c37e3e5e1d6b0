#!/bin/bash
# eager small-batch host-overhead check: optimizer / graph / DDP GPU tests, batch-32 (x3, 100
# steps) and batch-128 eager benches, and a cProfile of the batch-32 eager step
set -e
set -o pipefail
O=gpurun_out/${1:-small_eager}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sgd or adam or graph or ddp" > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 240 python -u bench.py --batch 32 --steps 100 --warmup 10 > $O/e_$r.log 2>&1
  echo "b32 eager $(grep -o '"value": [0-9.]*' $O/e_$r.log)"
done
timeout -k 10 240 python -u bench.py --batch 128 --steps 40 --warmup 5 > $O/e128.log 2>&1
echo "b128 eager $(grep -o '"value": [0-9.]*' $O/e128.log)"
DCP_AUTOTUNE=0 timeout -k 10 300 python -u -m cProfile -o $O/b32.prof bench.py --batch 32 --steps 40 --warmup 5 > $O/b32p.log 2>&1
echo prof done
