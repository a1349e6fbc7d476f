#!/bin/bash
# Round 4: the (F0,F1) NGC6440E 256x256 grid leg -- host profile (3 repetitions + cProfile)
# and a kernel trace of the same script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/prof_grid_host.py 256 > gpurun_out/grid_host.txt 2>&1 || exit $?
head -40 gpurun_out/grid_host.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profgrid -o run -- \
    python3 scripts/prof_grid_host.py 256 > gpurun_out/profgrid.log 2>&1 || exit $?
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/profgrid/run_kernel_stats.csv')))
for r in rows[:16]: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms')"
