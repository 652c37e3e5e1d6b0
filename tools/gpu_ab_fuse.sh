#!/bin/bash
# A/B of the plain BN+ReLU dgrad-epilogue fusion (EPI 3) on the headline and TResNet
set -e
O=gpurun_out/${1:-abf}; mkdir -p $O
for c in r50 r50b; do
  for m in masked none; do
    DCP_BN_FUSE=$m timeout -k 10 240 python -u bench.py --config ${c%b} --steps 40 --warmup 5 > $O/$c-$m.log 2>&1
    python -c "import json; d=json.loads(open('$O/$c-$m.log').read().strip().splitlines()[-1]); print('$c', '$m', d['value'], d['ms_per_step'])"
  done
done
