#!/bin/bash
# iteration check: table transport + graph capture + direct 3x3 conv tests, then eager/graph bench
set -e
O=gpurun_out/${1:-iter}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "table or graphed or conv3x3_direct or conv_fwd" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for b in 32 128; do
  for g in "" "--graph"; do
    timeout -k 10 180 python -u bench.py --batch $b --steps 30 --warmup 5 $g > $O/bench_b${b}${g}.log 2>&1 || { tail -20 $O/bench_b${b}${g}.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_b${b}${g}.log').read().strip().splitlines()[-1]); print('b$b', '$g', d['value'], d['ms_per_step'])"
  done
done
