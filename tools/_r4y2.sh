set -e -o pipefail
O=gpurun_out/r4y2; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/ddp_$r.log 2>&1
  tail -1 $O/ddp_$r.log
done
bash tools/gpu_round.sh r4y2 tests smoke bench
