#!/bin/bash
# Round 4 solve iteration: pytest -m gpu, the solve phases at 9 pulsars, the 9-pulsar step
# timeline and the PTA bench line with the emulated world sizes (no other legs).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 scripts/diag/ts_probe.py 9 > gpurun_out/ts9.txt 2>&1 || exit $?
head -4 gpurun_out/ts9.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 bench.py --npsr 9 --steps 30 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world '' --cold-start 0 \
    > gpurun_out/prof9.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof9/run_kernel_trace.csv > gpurun_out/timeline9.txt 2>&1 || true
head -40 gpurun_out/timeline9.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --cold-start 0 \
    > gpurun_out/bench_r4h.json 2> gpurun_out/bench_r4h.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_r4h.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])
p=d.get('predicted_strong'); print({k:(v.get('ms_per_step'), v.get('value')) for k,v in p.items() if k!='method'})"
exit $rc
