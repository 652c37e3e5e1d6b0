#!/bin/bash
# tests for the new variants, per-shape wgrad A/B, whole-step A/B of tuning env strings
set -e
O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or narrow or variants" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 512 --cfgs ",12=32,12=32;5=4,12=32;5=8" > $O/ab.txt 2>&1
tail -1 $O/ab.txt
for t in "" "13=32" "12=32" "12=32,5=4" ""; do
  DCP_TUNE="$t" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b.log 2>&1
  echo "tune=[$t] $(grep -o '"value": [0-9.]*' $O/b.log)"
done
