#!/bin/bash
# store-decoupled 1x1 kernel: numerics, then the per-shape A/B against the shipped choice, with ablations
set -o pipefail
T=${1:-s6}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "conv1x1_weight_stationary" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh $T "convabs=3,7,13:${2:-,tg_ps=1,tg_ps=1;ablate=4,tg_ps=1;ablate=1,tg_ps=1;ablate=8,tg_ps=1;ablate=12,tg_ps=1;ablate=15}"
