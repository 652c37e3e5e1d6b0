#!/bin/bash
# fused-stem tests + A/B of the headline bench with the fused stem off / on + profile with it on
set -e
O=gpurun_out/stemab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_stem or stem or s2d" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b_off.log 2>&1
DCP_FUSED_STEM=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b_on.log 2>&1
echo "off $(grep -o '"value": [0-9.]*' $O/b_off.log) on $(grep -o '"value": [0-9.]*' $O/b_on.log)"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
DCP_FUSED_STEM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1
echo stemab done
