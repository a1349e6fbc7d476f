#!/bin/bash
# The 68-pulsar step over repeated bench runs on one box: which part moves between the ~0.38 and
# ~0.41 ms modes (the instrumented per-kernel times beside the timed step).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for k in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 --emulate-world 0 > gpurun_out/bim_$k.json 2> gpurun_out/bim_$k.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/bim_$k.json')); km=d['roofline']['kernel_ms']
print('run $k', d['ms_per_step'], round(sum(v for k2, v in km.items() if k2 != 'gram_span'), 4), km)"
done
