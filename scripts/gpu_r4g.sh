#!/bin/bash
# Round 4 measurement: pytest -m gpu, the solve phases and the 9-pulsar step timeline, then
# the default bench line with every leg and the profile passes (scripts/gpu_final.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 scripts/diag/ts_probe.py 9 apply > gpurun_out/ts9.txt 2>&1 || exit $?
tail -6 gpurun_out/ts9.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 bench.py --npsr 9 --steps 30 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 \
    > gpurun_out/prof9.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof9/run_kernel_trace.csv > gpurun_out/timeline9.txt 2>&1 || true
head -40 gpurun_out/timeline9.txt
bash scripts/gpu_final.sh || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_default.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
p=d.get('predicted_strong'); print({k:(v.get('ms_per_step'), v.get('value')) for k,v in p.items() if k!='method'})
print(d.get('cold_start')); print(d.get('j0740')); print(d.get('c2')); print(d.get('grid'))"
exit $rc
