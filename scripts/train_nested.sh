#!/usr/bin/env bash
# NESTED/train.sh: Clothing1M ResNet-50, nested dropout (std 100), frozen BN, 10k warm-up iterations
NGPU=${NGPU:-1} exec "$(dirname "$0")/../train.sh" --workload nested --dataset Clothing1M --arch resnet50 \
  --train-dir "${TRAIN_DIR:-/data/clothing1m/train}" --val-dir "${VAL_DIR:-/data/clothing1m/val}" \
  --warmUpIter 10000 --lr 0.01 --batchsize 128 --nbEpoch 150 --nested 100 --out-dir "${OUT:-output/nested}" "$@"
