#!/bin/bash
# 16-byte optimizer step + 4-wide weight refresh: numerics (optimizer, weight prep, models), then the
# headline and R50 b32 graph against the previous library build (DCP_LIB), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s48}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_workloads_gpu.py -x -q --timeout 300 --timeout-method thread -k "sgd or adam or weight_prep or linear or model or resnet or graph" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
bash tools/lib_ab.sh ${1:-s48} ab/_dcp_kernels_prev.so
