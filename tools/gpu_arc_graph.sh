#!/bin/bash
set -e
O=gpurun_out/${1:-arcg}; mkdir -p $O
for g in "" "--graph"; do
  timeout -k 10 240 python -u bench.py --config arcface --steps 30 --warmup 5 $g > $O/arc$g.log 2>&1
  python -c "import json; d=json.loads(open('$O/arc$g.log').read().strip().splitlines()[-1]); print('arcface', '$g', d['value'], d['ms_per_step'])"
done
for b in 256; do
  for g in "" "--graph"; do
    timeout -k 10 240 python -u bench.py --config arcface --batch $b --steps 30 --warmup 5 $g > $O/arc_b$b$g.log 2>&1
    python -c "import json; d=json.loads(open('$O/arc_b$b$g.log').read().strip().splitlines()[-1]); print('arcface b$b', '$g', d['value'], d['ms_per_step'])"
  done
done
