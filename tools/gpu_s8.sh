#!/bin/bash
set -o pipefail
bash tools/gpu_s6.sh $1 ",tg_ps=1,tg_ps=1;ablate=4,tg_ps=1;ablate=8,tg_ps=1;ablate=12" || exit $?
DCP_TUNE=tg_ps=1 bash tools/gpu_round.sh ${1}pmc pmc6=3,13
