#!/bin/bash
# GPU tests, solve phase timestamps (fused-apply step), then the PTA step with the emulated shards.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 scripts/diag/ts_probe.py 9 apply > gpurun_out/ts9a.txt 2>&1 || exit $?
tail -6 gpurun_out/ts9a.txt
timeout -k 10 300 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || { tail -20 gpurun_out/bench_k.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_k.json')); p=d['predicted_strong']
print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (p[k]['ms_per_step'], p[k]['value']) for k in ('n1','n2','n4','n8')})"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 bench.py --npsr 9 --steps 40 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 \
    > gpurun_out/prof9.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof9/run_kernel_trace.csv > gpurun_out/timeline9.txt 2>&1 || true
tail -14 gpurun_out/timeline9.txt
