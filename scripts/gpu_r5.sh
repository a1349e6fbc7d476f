#!/bin/bash
# round-5 loop on the GPU box: the whole GPU test suite, then one bench line (extra bench
# arguments in $@; default all legs but the CPU baseline), summarised by scripts/bench_brief.py
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --cpu-baseline 0 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python scripts/bench_brief.py gpurun_out/bench.json
