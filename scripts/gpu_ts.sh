#!/bin/bash
# k_solve_dmx phase timestamps (workgroup 0) at 9 and 68 pulsars, the bench's fused-apply step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 scripts/diag/ts_probe.py 9 apply > gpurun_out/ts9a.txt 2>&1 || exit $?
timeout -k 10 120 python3 scripts/diag/ts_probe.py 68 apply > gpurun_out/ts68a.txt 2>&1 || exit $?
tail -6 gpurun_out/ts9a.txt; tail -6 gpurun_out/ts68a.txt
