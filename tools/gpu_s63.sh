#!/bin/bash
# stem backward: last k-step on 16-deep MFMAs. Numerics (stem / model tests), the kernel alone, then the
# headline (b4096) and b32 graph against the previous library build (DCP_LIB), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s63}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_large_batch_gpu.py -x -q --timeout 300 --timeout-method thread -k "stem or model or resnet" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
for lib in "" ab/_dcp_kernels_prev.so; do
  DCP_LIB=$lib timeout -k 10 200 python -u tools/stem_bwd_bench.py > $O/stem_$(basename ${lib:-new} .so).txt 2>&1 || exit 1
  echo "${lib:-new}: $(grep full $O/stem_$(basename ${lib:-new} .so).txt)"
done
bash tools/lib_ab.sh ${1:-s63} ab/_dcp_kernels_prev.so
