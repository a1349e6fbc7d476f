#!/bin/bash
# Iteration call on the GPU box: a pytest -m gpu selection ($1, default the parity files),
# a short bench line (PTA leg only) and a rocprofv3 kernel trace of it.  A fault, abort or
# time limit ends the call; test failures (rc 1) still run the bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${1:-"tests/test_gpu_parity.py tests/test_fullshape.py tests/test_gpu_stage.py"}
timeout -k 10 600 python -u -m pytest $SEL -m gpu --maxfail=20 -q -rf -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 bench.py --grid 0 --j0740 0 --cpu-baseline 0 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_iter.json')); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], r['kernel_ms']); print('C2', d.get('c2'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profi -o run -- \
    python3 bench.py --steps 20 --warmup 2 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 > gpurun_out/profi.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/profi | head -30
