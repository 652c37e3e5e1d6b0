#!/bin/bash
# per-GPU batch sweep of the secondary BASELINE.json configs
set -e
O=gpurun_out/bsweep; mkdir -p $O
IFS=, read -ra CBS <<< "${SWEEP:-r101 1024,resnext 256,tresnet 512,arcface 512,resnext 512}"
for cb in "${CBS[@]}"; do
  set -- $cb
  timeout -k 10 300 python -u bench.py --config $1 --batch $2 --steps 15 --warmup 4 > $O/bench_$1_b$2.log 2>&1
  echo "$1 b$2 $(grep -o '"value": [0-9.]*\|"max_mem_gb": [0-9.]*' $O/bench_$1_b$2.log | tr '\n' ' ')"
done
