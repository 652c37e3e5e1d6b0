#!/bin/bash
set -e
O=gpurun_out/${1:-rx}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grouped or resnext or parity" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 240 python -u bench.py --config resnext --steps 20 --warmup 5 > $O/bench_resnext.log 2>&1; tail -1 $O/bench_resnext.log
