#!/bin/bash
# Round measurements on the GPU box: hardware probes (FP64 MFMA rate, FP64 VALU issue and
# latency, MFMA/VALU co-issue, HBM copy), the default bench line, then scripts/gpu_prof.sh.
# Every GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 60 ./build/peaks > gpurun_out/peaks.json || exit $?
timeout -k 10 60 ./build/mfma_probe > gpurun_out/mfma_probe.json || exit $?
timeout -k 10 60 ./build/valu_probe > gpurun_out/valu_probe.txt || exit $?
timeout -k 10 60 ./build/coissue_probe > gpurun_out/coissue_probe.txt || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
bash scripts/gpu_prof.sh
