#!/bin/bash
# Tile / pipeline configuration A/B (tools/conv_bench.py --cfgs, interleaved in one process) and
# the headline step with the persistent tap GEMM switched on (DCP_TUNE 20=1).
set -e
set -o pipefail
O=gpurun_out/r3ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "persistent" > $O/ps_tests.log 2>&1 || { tail -30 $O/ps_tests.log; exit 1; }
tail -1 $O/ps_tests.log
timeout -k 10 900 python -u tools/conv_bench.py --batch 1024 --iters 10 --cfgs ",20=1,20=1;21=64,1=3;8=32,3=1,3=1;4=2" > $O/ab_all.txt 2>&1
tail -2 $O/ab_all.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log | grep -o '"value": [0-9.]*'
DCP_TUNE="20=1" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_ps.log 2>&1
tail -1 $O/bench_ps.log | grep -o '"value": [0-9.]*'
