#!/bin/bash
# One iteration on the GPU box: the GPU test suite, then the 9-pulsar step timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
bash scripts/gpu_timeline.sh ${1:-9} > gpurun_out/tl_iter.txt 2>&1 || { tail -20 gpurun_out/tl_iter.txt; exit 1; }
head -30 gpurun_out/tl_iter.txt
