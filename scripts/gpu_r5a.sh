#!/bin/bash
# round-5 check: the RCCL gather tests, then a short bench (PTA + grid + predicted strong scaling)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rccl.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/rccl.log 2>&1
echo "rccl rc=$?"; tail -6 gpurun_out/rccl.log
timeout -k 10 400 python bench.py --j0740 0 --c2 0 --cpu-baseline 0 > gpurun_out/b0.json 2> gpurun_out/b0.err || exit $?
python scripts/bench_brief.py gpurun_out/b0.json
