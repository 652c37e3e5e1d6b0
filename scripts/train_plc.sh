#!/usr/bin/env bash
# PLC: Clothing1M annotation-list data with LRT label correction
NGPU=${NGPU:-1} exec "$(dirname "$0")/../train.sh" --workload plc --data list --folder "${FOLDER:-/data/clothing1m}" --num-classes 14 "$@"
