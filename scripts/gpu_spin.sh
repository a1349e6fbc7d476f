#!/bin/bash
# The 68-pulsar step with and without a long active wait in the HIP runtime's host
# synchronisation (ROC_ACTIVE_WAIT_TIMEOUT, microseconds), alternating on one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for k in 1 2 3 4; do
  for w in default 2000; do
    if [ "$w" = default ]; then
      timeout -k 10 200 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 --emulate-world 0 > gpurun_out/spin.json 2> gpurun_out/spin.err || exit $?
    else
      ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 200 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 --emulate-world 0 > gpurun_out/spin.json 2> gpurun_out/spin.err || exit $?
    fi
    python3 -c "
import json; d=json.load(open('gpurun_out/spin.json')); print('wait $w', d['ms_per_step'])"
  done
done
