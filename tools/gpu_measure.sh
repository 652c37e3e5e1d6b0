#!/bin/bash
# One GPU-box measurement pass: three rocprofv3 PMC passes over a short headline run
# (MFMA busy / LDS conflicts / wave stalls, then HBM read, then HBM write bytes), every
# BASELINE.json config through bench.py, and the stock PyTorch-ROCm ResNet-50 step at the
# headline batch. Each GPU step has its own time limit; the chain stops at the first failure.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- bash tools/gpu_measure.sh [pmc|bench|stock]...
set -e
mkdir -p gpurun_out/meas
O=gpurun_out/meas
what="${*:-pmc bench stock}"
if [[ $what == *pmc* ]]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  PASS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PASS1 --output-format csv -d $O/pmc1 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc1.log 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc2.log 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc3 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc3.log 2>&1
fi
if [[ $what == *bench* ]]; then
  for c in r50 arcface resnext r101 tresnet; do
    timeout -k 10 240 python -u bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1
  done
fi
if [[ $what == *stock* ]]; then
  timeout -k 10 600 python -u tools/bench_torch_reference.py --batch 512 --warmup 3 > $O/stock_r50_b512.log 2>&1
fi
echo measure done
