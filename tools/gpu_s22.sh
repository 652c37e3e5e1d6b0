#!/bin/bash
# fused squeeze-excitation gate + adaptive BN-backward reduction grid: numerics, then TResNet-M b16 / R50 b32
# graph and the headline, fused vs GEMM chain (DCP_SE_FUSED=0), twice
set -o pipefail
O=gpurun_out/${1:-s22}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "se_gate or bn_bwd or tresnet or bn_fin_act or chan_scale or bn_" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_workloads_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t2.log 2>&1
rc=$?; tail -3 $O/t2.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "DCP_SE_FUSED=1" "DCP_SE_FUSED=0"; do
    tag=$([ "$cfg" = "DCP_SE_FUSED=1" ] && echo on || echo off)
    env $cfg timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
  done
  timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/r50b32_$r.log 2>&1 || exit 1
  echo "r50 b32 graph: $(grep -o '"value": [0-9.]*' $O/r50b32_$r.log)"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1024.log 2>&1 || exit 1
echo "r50 b1024: $(grep -o '"value": [0-9.]*' $O/b1024.log)"
timeout -k 10 300 python -u bench.py --config tresnet --steps 10 --warmup 3 > $O/tres1024.log 2>&1 || exit 1
echo "tresnet b1024-config: $(grep -o '"value": [0-9.]*' $O/tres1024.log)"
