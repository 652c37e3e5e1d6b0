#!/bin/bash
# headline A/B: split-K heuristic on vs off (it should not apply at batch 1024 but for the head), twice
set -o pipefail
O=gpurun_out/${1:-s28}; mkdir -p $O
for r in 1 2; do
  for cfg in "" "tg_split_k=2"; do
    tag=$([ -z "$cfg" ] && echo on || echo off)
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b1024 $tag: $(grep -o '"value": [0-9.]*' $O/b1024_${tag}_$r.log)"
  done
done
