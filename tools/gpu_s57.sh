#!/bin/bash
# per-GPU batch for the other BASELINE configs (288 GB sizing): arcface / resnext / tresnet
set -o pipefail
O=gpurun_out/${1:-s57}; mkdir -p $O
for cb in arcface:1024 arcface:2048 arcface:4096 resnext:1024 resnext:2048 resnext:3072 tresnet:1024 tresnet:2048 tresnet:4096; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 300 python -u bench.py --config $c --batch $b --steps 10 --warmup 4 > $O/${c}_b$b.log 2>&1 || exit 1
  echo "$c b$b: $(grep -o '"value": [0-9.]*' $O/${c}_b$b.log) $(grep -o '"max_mem_gb": [0-9.]*' $O/${c}_b$b.log)"
done
