#!/usr/bin/env bash
# BASELINE/train.sh equivalent: 2-GPU DDP + SyncBN, TResNet-M, batch 16/GPU
NGPU=${NGPU:-2} exec "$(dirname "$0")/../train.sh" --workload baseline --folder "${FOLDER:-/root/commonfile/foodH/}" --model "${MODEL:-tresnet_m}" --batchsize "${BS:-16}" "$@"
