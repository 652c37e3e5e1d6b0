#!/bin/bash
set -e
O=gpurun_out/gconv; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grouped" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config resnext --batch 512 --steps 12 --warmup 3 > $O/b_new.log 2>&1
DCP_TUNE="16=16" timeout -k 10 300 python -u bench.py --config resnext --batch 512 --steps 12 --warmup 3 > $O/b_old.log 2>&1
echo "new $(grep -o '"value": [0-9.]*' $O/b_new.log) old $(grep -o '"value": [0-9.]*' $O/b_old.log)"
