#!/bin/bash
# Round 4, second pass: pytest -m gpu (assertion failures reported, a crash / limit stops the
# run), the bench line, and a kernel trace of a 9-pulsar shard (the per-rank batch at 8 GPUs).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_r4b.json 2> gpurun_out/bench_r4b.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_r4b.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
p=d.get('predicted_strong'); print({k:(v.get('ms_per_step'), v.get('value')) for k,v in p.items() if k!='method'})
print(json.dumps(d.get('cold_start'))); print(json.dumps(d.get('j0740'))[:500]); print(json.dumps(d.get('c2'))[:300])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 bench.py --npsr 9 --steps 30 --warmup 5 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world '' --cold-start 0 \
    > gpurun_out/prof9.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof9/run_kernel_trace.csv > gpurun_out/timeline9.txt 2>&1 || true
head -40 gpurun_out/timeline9.txt
