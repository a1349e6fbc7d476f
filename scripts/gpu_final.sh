#!/bin/bash
# Round-6 final measurements on the GPU box: GPU tests, the default bench line (100 steps) and
# a 20-step line, the profile passes (scripts/gpu_prof.sh), the 9-pulsar step timeline and
# per-workgroup timeline.  Each GPU step has its own time limit; any failure stops it.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_final.log 2>&1 || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -2 gpurun_out/pytest_final.log
timeout -k 10 500 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 scripts/bench_brief.py gpurun_out/bench_default.json | cut -c1-400
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err || { tail -20 gpurun_out/bench_20.err; exit 1; }
python3 scripts/bench_brief.py gpurun_out/bench_20.json | head -2 | cut -c1-300
bash scripts/gpu_prof.sh > gpurun_out/prof_run.log 2>&1 || { tail -20 gpurun_out/prof_run.log; exit 1; }
tail -1 gpurun_out/prof_run.log
bash scripts/gpu_timeline.sh 9 > gpurun_out/tl_final.txt 2>&1 || { tail -20 gpurun_out/tl_final.txt; exit 1; }
head -16 gpurun_out/tl_final.txt
timeout -k 10 200 python3 scripts/diag/wg_timeline.py 9 5 > gpurun_out/wgt9.txt 2>&1 || { tail -20 gpurun_out/wgt9.txt; exit 1; }
cat gpurun_out/wgt9.txt
