#!/bin/bash
# the chunked-grid test, a two-rank rehearsal of the multi-rank bench on one GPU (gloo
# collectives; not a scaling measurement), then 20-step runs after 5 and 100 warm-up steps
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_stage.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "chunked or resident" > gpurun_out/pt_ch.log 2>&1
rc=$?; tail -3 gpurun_out/pt_ch.log; [ $rc -eq 0 ] || exit $rc
export PINT_BENCH_SHARE_GPU=1 PINT_BENCH_BACKEND=gloo
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/b2r.json 2> gpurun_out/b2r.err || { tail -20 gpurun_out/b2r.err; exit 1; }
tail -c 1500 gpurun_out/b2r.json
unset PINT_BENCH_SHARE_GPU PINT_BENCH_BACKEND
for w in 5 100 5 100; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup $w --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 \
     > gpurun_out/bw$w.json 2> gpurun_out/bw$w.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bw$w.json').read().strip().splitlines()[-1]);print('warmup $w', d['ms_per_step'])"
done
