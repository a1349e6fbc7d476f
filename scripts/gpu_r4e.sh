#!/bin/bash
# Round 4, small-batch pass: the diagonal-factor and rsq probes, host enqueue vs device time
# (direct vs HIP-graph steps) at 9 and 68 pulsars, per-call host timing at 9, the solve's
# phases at 9, a 9-pulsar kernel trace with its step timeline, then pytest -m gpu.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 bench/_bin/diag_probe > gpurun_out/diag_probe.txt 2>&1 || exit $?
timeout -k 10 60 bench/_bin/rsq_probe > gpurun_out/rsq_probe.txt 2>&1 || exit $?
cat gpurun_out/diag_probe.txt gpurun_out/rsq_probe.txt
timeout -k 10 200 python3 scripts/diag/graph_probe.py 9 > gpurun_out/graph9.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/diag/graph_probe.py 68 > gpurun_out/graph68.txt 2>&1 || exit $?
tail -2 gpurun_out/graph9.txt gpurun_out/graph68.txt
timeout -k 10 200 python3 scripts/host_timing.py 9 > gpurun_out/host9.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/diag/ts_probe.py 9 > gpurun_out/ts9.txt 2>&1 || exit $?
cat gpurun_out/host9.txt; tail -5 gpurun_out/ts9.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 bench.py --npsr 9 --steps 30 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world '' --cold-start 0 \
    > gpurun_out/prof9.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof9/run_kernel_trace.csv > gpurun_out/timeline9.txt 2>&1 || true
head -40 gpurun_out/timeline9.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
exit $rc
