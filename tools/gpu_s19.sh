#!/bin/bash
# fused BN finalize + apply (bn_fin_act): kernel numerics + model tests, then A/B against the two-launch
# path (DCP_BN_FIN_ACT=0) at the reference's small batches and the headline batch, twice
set -o pipefail
O=gpurun_out/${1:-s19}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "bn_fin_act or bn_act or iabn or batchnorm or bn_" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_workloads_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t2.log 2>&1
rc=$?; tail -3 $O/t2.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "DCP_BN_FIN_ACT=1" "DCP_BN_FIN_ACT=0"; do
    tag=$([ "$cfg" = "DCP_BN_FIN_ACT=1" ] && echo on || echo off)
    env $cfg timeout -k 10 300 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/r50b32_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b32 graph $tag: $(grep -o '"value": [0-9.]*' $O/r50b32_${tag}_$r.log)"
    env $cfg timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_${tag}_$r.log 2>&1 || exit 1
    echo "tresnet b16 graph $tag: $(grep -o '"value": [0-9.]*' $O/tres16_${tag}_$r.log)"
    env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${tag}_$r.log 2>&1 || exit 1
    echo "r50 b1024 $tag: $(grep -o '"value": [0-9.]*' $O/b1024_${tag}_$r.log)"
  done
done
