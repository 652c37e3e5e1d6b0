#!/bin/bash
# larger per-GPU batches for the configs still gaining at their defaults (ArcFace 112 px, TResNet-M)
set -o pipefail
O=gpurun_out/${1:-s61}; mkdir -p $O
for cb in arcface:4096 arcface:8192 arcface:16384 tresnet:4096 tresnet:8192; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 400 python -u bench.py --config $c --batch $b --steps 10 --warmup 4 > $O/${c}_b$b.log 2>&1 || exit 1
  echo "$c b$b: $(grep -o '"value": [0-9.]*' $O/${c}_b$b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_b$b.log) $(grep -o '"max_mem_gb": [0-9.]*' $O/${c}_b$b.log)"
done
