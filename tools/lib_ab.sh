#!/bin/bash
# Same-box A/B of the in-tree kernel library against other builds of it (DCP_LIB), interleaved:
#   /usr/local/graft/bin/gpurun -- bash tools/lib_ab.sh <tag> ab/_dcp_kernels_old.so [more.so ...]
# (build a variant by compiling the changed csrc file into an object and linking it with the
# other objects of ddp_classification_pytorch_amd/_build; ab/ is git-ignored scratch)
set -e
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
for r in 1 2; do
  for lib in "" "$@"; do
    n=$(basename "${lib:-in-tree}" .so)
    DCP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${n}_$r.log 2>&1
    echo "b1024 $n $(grep -o '"value": [0-9.]*' $O/b1024_${n}_$r.log)"
    DCP_LIB=$lib timeout -k 10 200 python -u bench.py --batch 32 --graph --steps 60 --warmup 5 > $O/b32_${n}_$r.log 2>&1
    echo "b32g $n $(grep -o '"value": [0-9.]*' $O/b32_${n}_$r.log)"
  done
done
