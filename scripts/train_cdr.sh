#!/usr/bin/env bash
# CDR/train.sh: single process, lr 0.1, batch 128
NGPU=${NGPU:-1} exec "$(dirname "$0")/../train.sh" --workload cdr --folder "${FOLDER:-/root/commonfile/food/}" --lr 0.1 --batch_size 128 --noise_rate 0.2 "$@"
