#!/bin/bash
# Quick bench: the PTA leg and the predicted strong scaling only (no grid / J0740 / C2 / CPU
# baseline / cold start); the JSON line to gpurun_out/benchq.json, a brief to stdout.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps ${STEPS:-100} --warmup ${WARM:-10} --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 "$@" \
    > gpurun_out/benchq.json 2> gpurun_out/benchq.err || { tail -20 gpurun_out/benchq.err; exit 1; }
grep -v "^\[trace\]" gpurun_out/benchq.err | tail -12
python3 scripts/bench_brief.py gpurun_out/benchq.json
