#!/bin/bash
# The 68-pulsar step over repeated bench runs (measured in round 4 with gc.disable() around the
# timed steps in bench.py: no change to the run-to-run spread, so bench.py leaves the collector on).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for k in 1 2 3 4 5 6; do
  timeout -k 10 200 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 --emulate-world 0 > gpurun_out/gc.json 2> gpurun_out/gc.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/gc.json')); print('gc-off run $k', d['ms_per_step'])"
done
