#!/bin/bash
# SE gate loads-first MFMA helper + bf16 channel-scale gate gradient: numerics, TResNet-M b16 graph
set -o pipefail
O=gpurun_out/${1:-s30}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "se_gate or hw_reductions or pools or tresnet or chan" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_workloads_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t2.log 2>&1
rc=$?; tail -2 $O/t2.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config tresnet --batch 16 --graph --steps 60 --warmup 5 > $O/tres16_$r.log 2>&1 || exit 1
  echo "tresnet b16 graph: $(grep -o '"value": [0-9.]*' $O/tres16_$r.log)"
done
