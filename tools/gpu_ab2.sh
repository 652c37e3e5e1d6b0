#!/bin/bash
# GPU tests matching $1, then an in-process per-shape A/B of tuning configs $2 (tools/conv_bench.py --cfgs)
set -e
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 512 --cfgs "$2" > $O/ab.txt 2>&1
tail -1 $O/ab.txt
