#!/bin/bash
# One GPU call: pytest -m gpu (selection $1, default all of tests/), then the default bench
# line.  Test failures (pytest rc 1) still run the bench; anything else -- a fault, an abort,
# a time limit -- ends the call there.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu --maxfail=30 -q -rf -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_check.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_check.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 420 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
brc=$?
tail -3 gpurun_out/bench_default.err
exit $brc
