#!/bin/bash
# channel-major k order A/B: 3x3 tap-GEMM numerics, then conv_bench on the 3x3 shapes for the in-tree
# build and the tap-major build (ab/_dcp_kernels_tapmajor.so), interleaved twice, then the headline
set -o pipefail
O=gpurun_out/${1:-s14}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_autotune_variants_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
[ $rc -eq 0 ] || echo "(tests failed: measuring anyway)"
for r in 1 2; do
  for lib in "" ab/_dcp_kernels_tapmajor.so; do
    n=$(basename "${lib:-in-tree}" .so)
    DCP_LIB=$lib timeout -k 10 400 python -u tools/conv_bench.py --batch 1024 --iters 10 --no-miopen --only 2,6,10,12,16,18,22 > $O/cb_${n}_$r.txt 2>&1 || exit 1
    echo "$n $r: $(grep 'per-step totals' $O/cb_${n}_$r.txt)"
  done
done
for r in 1 2; do
  for lib in "" ab/_dcp_kernels_tapmajor.so; do
    n=$(basename "${lib:-in-tree}" .so)
    DCP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b1024_${n}_$r.log 2>&1 || exit 1
    echo "b1024 $n $(grep -o '"value": [0-9.]*' $O/b1024_${n}_$r.log)"
  done
done
