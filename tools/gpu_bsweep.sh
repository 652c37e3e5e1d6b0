#!/bin/bash
# headline batch sweep (final build)
set -e
O=gpurun_out/${1:-bsweep}; mkdir -p $O
for b in 128 256 512 1024 2048; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 20 --warmup 5 > $O/b$b.log 2>&1
  python -c "import json; d=json.loads(open('$O/b$b.log').read().strip().splitlines()[-1]); print('r50 b$b', d['value'], d['ms_per_step'], d['config']['max_mem_gb'])"
done
