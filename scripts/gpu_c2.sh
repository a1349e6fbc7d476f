#!/bin/bash
# C2 iteration on the GPU box: the ECORR / compact-layout tests, a bench line with the C2 leg
# (small PTA leg), and a kernel trace of the C2 leg.  Any failure ends the call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage.py tests/test_gpu_parity.py -m gpu -k "b1855 or ecorr or compact" \
    -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_c2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- \
    python3 bench.py --steps 4 --warmup 1 --npsr 4 --grid 0 --j0740 0 --cpu-baseline 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2', d['c2'])"
python3 scripts/kstats.py gpurun_out/prof_c2 | head -24
