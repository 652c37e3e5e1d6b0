#!/bin/bash
# Batch-size sweep of the headline bench + per-shape conv timings at the headline batch.
set -e
O=gpurun_out/sweep; mkdir -p $O
for b in 128 192 256 384 512 640; do
  timeout -k 10 150 python -u bench.py --steps 12 --warmup 4 --batch $b > $O/bench_b$b.log 2>&1
  echo "b=$b $(grep -o '"value": [0-9.]*' $O/bench_b$b.log)" | tee -a $O/summary.txt
done
timeout -k 10 300 python -u tools/conv_bench.py --batch 512 --no-miopen > $O/conv_b512.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof128 -o run -- python3 -u bench.py --steps 6 --warmup 2 --batch 128 > $O/prof128.log 2>&1
echo sweep done
