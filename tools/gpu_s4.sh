#!/bin/bash
# ArcFace fused head: tests, bench, per-kernel profile
O=gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_arcface_fused_gpu.py tests/test_kernels_gpu.py -k "arcface" -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc ;; esac
timeout -k 10 200 python -u tools/arcface_bench.py > $O/arc_bench.txt 2>&1 || exit $?
cat $O/arc_bench.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/arcprof -o run -- python3 -u tools/arcface_bench.py --classes 10000 --mode fused --iters 20 > $O/arcprof.log 2>&1 || exit $?
python3 tools/rocpd_summary.py $O/arcprof/run_results.db --steps 24 --top 25 > $O/arcprof_summary.txt 2>&1
cat $O/arcprof_summary.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/arcprofu -o run -- python3 -u tools/arcface_bench.py --classes 10000 --mode unfused --iters 20 > $O/arcprofu.log 2>&1 || exit $?
python3 tools/rocpd_summary.py $O/arcprofu/run_results.db --steps 24 --top 25 > $O/arcprofu_summary.txt 2>&1
cat $O/arcprofu_summary.txt
