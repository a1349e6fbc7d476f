#!/bin/bash
# Round-6 iteration: GPU tests, 9-pulsar timeline + solve phases, per-workgroup timeline, the
# grid leg's host profile.  Each GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
bash scripts/gpu_timeline.sh 9 > gpurun_out/tl_iter.txt 2>&1 || { tail -20 gpurun_out/tl_iter.txt; exit 1; }
head -16 gpurun_out/tl_iter.txt; tail -9 gpurun_out/tl_iter.txt
timeout -k 10 200 python3 scripts/diag/wg_timeline.py 9 5 > gpurun_out/wgt9.txt 2>&1 || { tail -20 gpurun_out/wgt9.txt; exit 1; }
cat gpurun_out/wgt9.txt
timeout -k 10 200 python3 scripts/prof_grid_host.py 256 3 > gpurun_out/grid_host.txt 2>&1 || { tail -20 gpurun_out/grid_host.txt; exit 1; }
head -45 gpurun_out/grid_host.txt
timeout -k 10 200 python3 scripts/diag/wg_timeline.py 68 3 > gpurun_out/wgt68.txt 2>&1 || { tail -20 gpurun_out/wgt68.txt; exit 1; }
cat gpurun_out/wgt68.txt
for b in 1024 512 256; do
    timeout -k 10 60 ./bench/_bin/diag_probe_$b > gpurun_out/diag_$b.txt 2>&1 || { tail -20 gpurun_out/diag_$b.txt; exit 1; }
    cat gpurun_out/diag_$b.txt
done
