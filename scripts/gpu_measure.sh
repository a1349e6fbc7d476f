#!/bin/bash
# Round measurements without the hardware probes (their figures stay in profiles/peaks_*.json):
# the default bench line, then scripts/gpu_prof.sh's kernel trace and PMC passes.  Every GPU
# step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('BENCH', d['value'], d['ms_per_step'])"
bash scripts/gpu_prof.sh
