#!/bin/bash
# Grid leg: host profile over 8 grids (current tree), then bench.py's grid leg alone.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/prof_grid_host.py 256 8 > gpurun_out/grid_host.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 > gpurun_out/bench_grid.json 2> gpurun_out/bench_grid.err || exit $?
cat gpurun_out/grid_host.txt | head -45
python3 -c "import json; print(json.load(open('gpurun_out/bench_grid.json'))['grid'])"
