#!/bin/bash
# SE gate kernels with the weight fragments loaded at entry + 8-wide staging: numerics, then TResNet-M
# small-batch HIP-graph steps against the previous library build (DCP_LIB), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s45}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "se_gate or tresnet or chan_scale" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in "" "ab/_dcp_kernels_prev.so"; do
    tag=$([ -z "$lib" ] && echo new || echo prev)
    for b in 16 32; do
      DCP_LIB=$lib timeout -k 10 300 python -u bench.py --config tresnet --batch $b --graph --steps 60 --warmup 5 > $O/tres${b}_${tag}_$r.log 2>&1 || exit 1
      echo "tresnet b$b graph $tag: $(grep -o '"value": [0-9.]*' $O/tres${b}_${tag}_$r.log)"
    done
  done
done
