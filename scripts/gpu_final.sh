#!/bin/bash
# Round-end measurement on the GPU box: the default bench line (all legs), then
# scripts/gpu_prof.sh (kernel stats, C2 trace, HBM and Gram PMC passes).  Each GPU step has
# its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
bash scripts/gpu_prof.sh
