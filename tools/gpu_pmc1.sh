#!/bin/bash
# GPU tests ($1 filter), bench, and PMC pass 1 (MFMA busy, LDS bank conflicts, wave-cycle split)
set -e
O=gpurun_out/pmcq; mkdir -p $O
if [ -n "$1" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
grep -o '"value": [0-9.]*' $O/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PASS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PASS1 --output-format csv -d $O/pmc1 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc1.log 2>&1
echo pmc done
