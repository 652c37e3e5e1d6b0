set -e
O=gpurun_out/ablate; mkdir -p $O
timeout -k 10 600 python -u tools/conv_bench.py --batch 512 --cfgs ",2=1,2=2,2=3" > $O/ablate_b512.txt 2>&1
echo done
