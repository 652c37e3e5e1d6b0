#!/bin/bash
# folded InplaceABN weight: numerics, then the reference default config (TResNet-M batch 16, HIP
# graph) and R50 batch 32 with the fold on vs off, twice
set -o pipefail
O=gpurun_out/${1:-s16}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_workloads_gpu.py -x -v --timeout 200 --timeout-method thread -k "iabn or linear or tresnet or inplace" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "" "DCP_IABN_FOLD=0"; do
    tag=$([ -z "$cfg" ] && echo on || echo off)
    env $cfg timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
    env $cfg timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 60 --warmup 5 > $O/r50b32_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b32 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b32_${tag}_$r.log)"
  done
done
