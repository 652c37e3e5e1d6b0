#!/bin/bash
# Run one gpurun call, retrying ONLY while gpurun reports "no box / slot free" (exit 3: nothing ran,
# nothing charged).  Any other outcome -- success, a failed or timed-out GPU step -- ends it.
#   tools/gpurun_retry.sh <timeout_s> <command...>
t=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_retry] no slot free (attempt $i); retrying in 120 s"
  sleep 120
done
exit 3
