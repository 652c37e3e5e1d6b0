#!/bin/bash
# split-K net width A/B: heuristic vs tg_split_k=1 (grids < 2 rounds, slices >= 4 units), small batches, twice
set -o pipefail
O=gpurun_out/${1:-s37}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "split_k" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "" "tg_split_k=1"; do
    tag=$([ -z "$cfg" ] && echo base || echo oneround)
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/r50b32_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b32 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b32_${tag}_$r.log)"
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --batch 64 --graph --steps 60 --warmup 5 > $O/r50b64_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b64 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b64_${tag}_$r.log)"
    DCP_TUNE=$cfg timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
  done
done
