#!/bin/bash
# BN / reduction kernels check: their GPU tests, then tools/gpu_tune_check.sh's benches
set -e
set -o pipefail
T=${1:-bn_check}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or stats or sync or reduce or graph" > $O/tests.log 2>&1
tail -1 $O/tests.log
bash tools/gpu_tune_check.sh $T
