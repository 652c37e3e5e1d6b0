#!/bin/bash
# session-6 GPU call: new-kernel tests, then the ArcFace head and 1x1 weight-stationary A/B
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1300 python -u -m pytest tests/test_kernels_gpu.py -k "weight_stationary or arcface" tests/test_arcface_fused_gpu.py tests/test_autotune_variants_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -v -s --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -25 $O/t.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc ;; esac
timeout -k 10 200 python -u tools/arcface_bench.py > $O/arc_bench.txt 2>&1 || exit $?
cat $O/arc_bench.txt
timeout -k 10 600 python -u tools/conv_bench.py --batch 1024 --iters 10 --only 3,4,7,9,13,15 --cfgs ",tg_ws=1" > $O/ws_ab.txt 2>&1 || exit $?
cat $O/ws_ab.txt
