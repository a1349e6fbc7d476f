#!/bin/bash
# Host-side helper: run one gpurun call, re-submitting it only while gpurun reports that
# nothing ran (rc 3: no box or slot free; or a box that stopped responding while being
# prepared -- "transient", nothing charged), at most N times (default 12), 1 minute apart.
#   scripts/gpurun_retry.sh LOG TIMEOUT 'command' [N]
LOG=$1; TO=$2; CMD=$3; N=${4:-12}
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  echo "[retry $i: rc $rc]" >> "$LOG.retries"
  sleep 60
done
exit 3
