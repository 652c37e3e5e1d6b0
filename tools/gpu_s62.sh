#!/bin/bash
# b4096 headline: BN-apply nontemporal stores (bn_act_variant=1) and 8 rows per thread (ew_rows=8) vs default,
# interleaved twice
set -o pipefail
O=gpurun_out/${1:-s62}; mkdir -p $O
for r in 1 2; do
  for v in "" "bn_act_variant=1" "ew_rows=8"; do
    tag=${v:-default}; tag=${tag%%=*}
    DCP_TUNE=$v timeout -k 10 300 python -u bench.py > $O/b4096_${tag}_$r.log 2>&1 || exit 1
    echo "b4096 ${v:-default}: $(grep -o '"value": [0-9.]*' $O/b4096_${tag}_$r.log)"
  done
done
