#!/bin/bash
# split-K of the 128-row tap GEMM at short grids: numerics (new tests + every conv / autotune test), then
# R50 b32 / b16 / TResNet b16 graph on vs off (DCP_TUNE=tg_split_k=2) twice, and the headline
set -o pipefail
O=gpurun_out/${1:-s27}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_autotune_variants_gpu.py -x -v --timeout 300 --timeout-method thread -k "split_k or conv or autotune or linear or big or variant or candidate" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "" "tg_split_k=2"; do
    tag=$([ -z "$cfg" ] && echo on || echo off)
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/r50b32_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b32 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b32_${tag}_$r.log)"
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --batch 16 --graph --steps 100 --warmup 5 > $O/r50b16_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b16_${tag}_$r.log)"
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1024.log 2>&1 || exit 1
echo "r50 b1024: $(grep -o '"value": [0-9.]*' $O/b1024.log)"
