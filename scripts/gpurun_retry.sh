#!/bin/bash
# Host-side helper: run one gpurun call, re-submitting it only while gpurun answers 3 (no box
# or slot free: nothing ran, nothing charged), at most 12 times, 2 minutes apart.
#   scripts/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry $i: rc 3]" >> "$LOG.retries"
  sleep 120
done
exit 3
