set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2a/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > gpurun_out/r2a/prof.log 2>&1
echo rc=$?
