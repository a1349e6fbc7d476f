#!/bin/bash
# Round-4 check on the GPU box: pytest -m gpu (assertion failures are reported and the run goes
# on; a crash, abort or time limit stops it), then the driver's bench command line (with the
# emulated world sizes and the cold start), then the host profile of the single fits.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_r4.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
print(json.dumps(d.get('predicted_strong'))); print(json.dumps(d.get('cold_start')))
print(json.dumps(d.get('j0740'))[:600]); print(json.dumps(d.get('c2'))[:400])"
timeout -k 10 300 python3 scripts/diag/fit_profile.py > gpurun_out/fit_profile.txt 2>&1 || exit $?
grep "==" gpurun_out/fit_profile.txt
timeout -k 10 120 python3 scripts/host_timing.py 9 > gpurun_out/host_timing9.txt 2>&1 || exit $?
tail -3 gpurun_out/host_timing9.txt
