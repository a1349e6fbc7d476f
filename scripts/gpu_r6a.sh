#!/bin/bash
# Round-6 iteration: GPU tests, 9-pulsar timeline, per-workgroup timelines (9 and 68 pulsars),
# a Gram N-split sweep at 9 pulsars, then the default bench line.  Each GPU step has its own
# time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
bash scripts/gpu_timeline.sh 9 > gpurun_out/tl_iter.txt 2>&1 || { tail -20 gpurun_out/tl_iter.txt; exit 1; }
head -24 gpurun_out/tl_iter.txt
timeout -k 10 200 python3 scripts/diag/wg_timeline.py 9 5 > gpurun_out/wgt9.txt 2>&1 || { tail -20 gpurun_out/wgt9.txt; exit 1; }
cat gpurun_out/wgt9.txt
timeout -k 10 200 python3 scripts/diag/wg_timeline.py 68 5 > gpurun_out/wgt68.txt 2>&1 || { tail -20 gpurun_out/wgt68.txt; exit 1; }
cat gpurun_out/wgt68.txt
bash scripts/gpu_sweep.sh PINT_NSPLIT "28 14" 9 > gpurun_out/sweep_nsplit.txt 2>&1 || { tail -20 gpurun_out/sweep_nsplit.txt; exit 1; }
grep -A3 "==\|span" gpurun_out/sweep_nsplit.txt | head -20
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r06a.json 2> gpurun_out/bench_r06a.err || { tail -20 gpurun_out/bench_r06a.err; exit 1; }
python3 scripts/bench_brief.py gpurun_out/bench_r06a.json 2>/dev/null || head -c 1500 gpurun_out/bench_r06a.json
