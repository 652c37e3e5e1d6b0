#!/usr/bin/env bash
# torchrun launcher (replaces the reference's `python -m torch.distributed.launch
# --nproc_per_node=2 main.py --world_size=2`, BASELINE/train.sh:1).
#
#   NGPU=8 ./train.sh --workload baseline --folder /data/foodH --model resnet50 --batchsize 64
#   NGPU=2 ./train.sh --workload arcface --folder /data/foodH
#   NGPU=1 ./train.sh --workload cdr --folder /data/food --lr 0.1 --batch_size 128
#
# One process per GPU over RCCL (torch.distributed backend "nccl" on ROCm).
set -euo pipefail
NGPU=${NGPU:-2}
PORT=${MASTER_PORT:-29500}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
if [ -n "${GPUS:-}" ]; then export HIP_VISIBLE_DEVICES="$GPUS"; fi
if [ "$NGPU" -le 1 ]; then
  exec python "$HERE/main.py" "$@"
fi
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
  --master-port "$PORT" "$HERE/main.py" --world_size "$NGPU" "$@"
