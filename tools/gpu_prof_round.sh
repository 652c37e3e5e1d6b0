#!/bin/bash
# Round measurement pass: rocprofv3 kernel trace of the headline step, native shard-loader
# throughput, and every BASELINE.json config through bench.py.  Each GPU step has its own
# time limit; the chain stops at the first failure.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- bash tools/gpu_prof_round.sh <tag> [prof] [loader] [bench]
set -e
T=${1:-r2}; shift || true
O=gpurun_out/$T; mkdir -p $O
what="${*:-prof loader bench}"
if [[ $what == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1
  echo prof done; tail -1 $O/prof.log
fi
if [[ $what == *loader* ]]; then
  timeout -k 10 300 python -u tools/loader_bench.py --images 4096 --batch 512 --threads 16 --epochs 3 > $O/loader.log 2>&1
  tail -1 $O/loader.log
fi
if [[ $what == *bench* ]]; then
  for c in r50 arcface resnext r101 tresnet; do
    timeout -k 10 240 python -u bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1
    tail -1 $O/bench_$c.log
  done
fi
echo measure done
