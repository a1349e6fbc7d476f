#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats.  Each GPU step has its
# own time limit; a crash/timeout/abort (anything but pytest's "tests failed" status 1)
# ends the script before the next GPU step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <allowed-nonzero> <cmd...>
    local name=$1 ok=$2; shift 2
    echo "== $name: $*" >> gpurun_out/steps.log
    "$@"
    local rc=$?
    echo "== $name rc=$rc" >> gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ "$rc" != "$ok" ]; then exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest 1 timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1
    tail -30 gpurun_out/pytest_gpu.log
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 0 timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
    cat gpurun_out/bench.json
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
        -o run -- python3 bench.py --steps 10 --warmup 2 --grid 64 --j0740 0 --cpu-baseline 0 \
        > gpurun_out/prof.log 2>&1
    step pmc 0 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch \
        -o run -- python3 bench.py --steps 2 --warmup 1 --grid 0 --j0740 0 --cpu-baseline 0 \
        > gpurun_out/pmc_fetch.log 2>&1
    step pmc2 0 timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write \
        -o run -- python3 bench.py --steps 2 --warmup 1 --grid 0 --j0740 0 --cpu-baseline 0 \
        > gpurun_out/pmc_write.log 2>&1
fi
if [ "$MODE" = profj ]; then  # the J0740 legs (C3 Downhill, (M2,SINI) grid) on their own
    step rocprofj 0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profj \
        -o run -- python3 bench.py --steps 1 --warmup 1 --npsr 1 --grid 0 --j0740 256 --cpu-baseline 0 \
        > gpurun_out/profj.log 2>&1
fi
if [ "$MODE" = all ] || [ "$MODE" = peaks ]; then
    step peaks 0 timeout -k 10 120 ./build/peaks > gpurun_out/peaks.json
    cat gpurun_out/peaks.json
fi
cat gpurun_out/steps.log
echo done
