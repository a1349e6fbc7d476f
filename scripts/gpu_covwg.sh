#!/bin/bash
# A/B of k_cov_dmx's workgroups per instance on the 68-pulsar step: the default cap (1 at 68
# pulsars) against PINT_COV_WG=3, alternating on one box, the bench's default step count.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in 0 3 0 3 0 3; do
  PINT_COV_WG=$w timeout -k 10 300 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 --emulate-world 0 > gpurun_out/covwg_$w.json 2> gpurun_out/covwg_$w.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/covwg_$w.json'))
print('cov_wg $w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'].get('k_eval_M'))"
done
