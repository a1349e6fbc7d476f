#!/bin/bash
# Host-side helper: run one gpurun call, re-submitting it only while gpurun answers 3 (no box
# or slot free: nothing ran, nothing charged), at most N times (default 12), 2 minutes apart.
#   scripts/gpurun_retry.sh LOG TIMEOUT 'command' [N]
LOG=$1; TO=$2; CMD=$3; N=${4:-12}
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry $i: rc 3]" >> "$LOG.retries"
  sleep 120
done
exit 3
