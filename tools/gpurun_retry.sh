#!/bin/bash
# Run one gpurun call, retrying ONLY while nothing ran on a GPU: exit 3 (no box / slot free) or a
# "status=transient" verdict whose run time is 0 (the box failed while being prepared; nothing
# charged).  Any other outcome -- success, a failed or timed-out GPU step -- ends it.
#   tools/gpurun_retry.sh <timeout_s> <command...>
t=$1; shift
log=$(mktemp)
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1 | tee "$log"
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 3 ] && ! grep -q "status=transient.*run 0.0s" "$log"; then rm -f "$log"; exit $rc; fi
  echo "[gpurun_retry] nothing ran (rc $rc, attempt $i); retrying in 60 s"
  sleep 60
done
rm -f "$log"
exit 3
