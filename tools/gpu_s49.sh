#!/bin/bash
# plain BN + ReLU backward reduction in the dgrad epilogue at the headline batch: default (stage 4 only)
# vs stages 3-4 (DCP_BN_FUSE_PLAIN_MAX=2^26) vs every layer (DCP_BN_FUSE=all), interleaved twice
set -o pipefail
O=gpurun_out/${1:-s49}; mkdir -p $O
for r in 1 2; do
  for v in "X=0" "DCP_BN_FUSE_PLAIN_MAX=67108864" "DCP_BN_FUSE=all"; do
    tag=${v%%=*}
    env $v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${tag}_$r.log 2>&1 || exit 1
    echo "b1024 $v: $(grep -o '"value": [0-9.]*' $O/b1024_${tag}_$r.log)"
  done
done
