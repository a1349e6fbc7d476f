#!/bin/bash
# the whole GPU test suite, smoke(), then the grid leg alone twice
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep -E "FAILED" gpurun_out/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 scripts/grid_run.py 256 > gpurun_out/gf$i.json || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/gf$i.json'));print(d['value'], d['seconds_all'])"
done
