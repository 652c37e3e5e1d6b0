set -e
mkdir -p gpurun_out/it5
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or bn or mask" > gpurun_out/it5/tests.log 2>&1 || { tail -30 gpurun_out/it5/tests.log; exit 1; }
tail -1 gpurun_out/it5/tests.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > gpurun_out/it5/bench.log 2>&1
grep -o '"value": [0-9.]*' gpurun_out/it5/bench.log
timeout -k 10 300 python -u tools/epi_bench.py "" > gpurun_out/it5/epi.txt 2>&1
timeout -k 10 600 python -u tools/conv_bench.py --batch 512 --cfgs ",1=2;8=32,1=3;8=32" > gpurun_out/it5/ab.txt 2>&1
tail -1 gpurun_out/it5/ab.txt
