#!/bin/bash
# bandwidth probe + stem tests + forward-conv epilogue timings + headline bench
set -e
O=gpurun_out/fwd; mkdir -p $O
timeout -k 10 200 python -u tools/bw_probe.py > $O/bw.txt 2>&1
cat $O/bw.txt
bash tools/gpu_fwd.sh "${1:-stem}"
