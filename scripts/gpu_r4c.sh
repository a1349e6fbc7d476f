#!/bin/bash
# Round 4, third pass: the rsqrt probe (Cholesky pivot cost), the solve's phase timestamps at
# 9 and 68 pulsars, pytest -m gpu, and a short bench line (cold start with the staged upload).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out build
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 bench/rsq_probe.hip -o build/rsq_probe > /dev/null 2>&1 || exit 1
timeout -k 10 60 ./build/rsq_probe > gpurun_out/rsq_probe.txt 2>&1 || exit $?
cat gpurun_out/rsq_probe.txt
timeout -k 10 200 python3 scripts/diag/ts_probe.py 9 > gpurun_out/ts9.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/diag/ts_probe.py 68 > gpurun_out/ts68.txt 2>&1 || exit $?
tail -5 gpurun_out/ts9.txt; tail -5 gpurun_out/ts68.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world '' \
    > gpurun_out/bench_r4c.json 2> gpurun_out/bench_r4c.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_r4c.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms']); print(d['cold_start'])"
