#!/bin/bash
# 16-column narrow split reduction (BN-backward sums over more workgroups): numerics, then small batches + headline
# against the previous library build (DCP_LIB), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s43}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread -k "bn or syncbn or stats or split or reduc or tresnet or model or dgrad" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in "" "ab/_dcp_kernels_prev.so"; do
    tag=$([ -z "$lib" ] && echo new || echo prev)
    DCP_LIB=$lib timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/r50b32_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b32 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b32_${tag}_$r.log)"
    DCP_LIB=$lib timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
    DCP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b1024 $tag: $(grep -o '"value": [0-9.]*' $O/b1024_${tag}_$r.log)"
  done
done
