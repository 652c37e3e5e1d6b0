#!/bin/bash
# In-process per-shape A/B of kernel tuning configs (tools/conv_bench.py --cfgs "$1")
set -e
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python -u tools/conv_bench.py --batch 512 --cfgs "$1" > $O/ab_${2:-x}.txt 2>&1
tail -1 $O/ab_${2:-x}.txt
