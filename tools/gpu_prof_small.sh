#!/bin/bash
# rocprofv3 kernel statistics of the ResNet-50 batch-32 HIP-graph step (bench.py defaults)
set -e
set -o pipefail
O=gpurun_out/${1:-prof_small}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --batch ${2:-32} --graph --steps ${3:-20} --warmup 5 > $O/prof.log 2>&1
tail -1 $O/prof.log
