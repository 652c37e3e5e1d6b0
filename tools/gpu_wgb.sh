#!/bin/bash
set -e
O=gpurun_out/wg; mkdir -p $O
timeout -k 10 300 python -u tools/wgrad_bench.py > $O/wgrad_bench.txt 2>&1
cat $O/wgrad_bench.txt
