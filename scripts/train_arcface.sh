#!/usr/bin/env bash
# ARCFACE/arc_train.sh (HPC variant: BS=64)
NGPU=${NGPU:-2} exec "$(dirname "$0")/../train.sh" --workload arcface --folder "${FOLDER:-/root/commonfile/foodH/}" --batchsize "${BS:-32}" --optimizer "${OPT:-Adam}" "$@"
