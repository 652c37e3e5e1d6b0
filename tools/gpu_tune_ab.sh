mkdir -p gpurun_out/tune
for t in "" "1=3" "1=4" "0=64" "3=1" "1=3,3=1"; do
  DCP_TUNE="$t" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > "gpurun_out/tune/b_${t//[=,]/_}.log" 2>&1 || exit 1
  echo "$t $(grep -o '"value": [0-9.]*' gpurun_out/tune/b_${t//[=,]/_}.log)" | tee -a gpurun_out/tune/summary.txt
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "finalize" -x -q --timeout 120 --timeout-method thread > gpurun_out/tune/t.log 2>&1
