#!/bin/bash
# k_solve_dmx phase timestamps (ts_probe.py) and a kernel trace with k_greduce split into its
# Gram-element and DMX-bin launches (PINT_GREDUCE_SPLIT), both on the bench PTA.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/diag/ts_probe.py > gpurun_out/ts_probe.txt 2>&1 || exit $?
PINT_GREDUCE_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profg -o run -- \
    python3 bench.py --steps 20 --warmup 2 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 > gpurun_out/profg.log 2>&1
