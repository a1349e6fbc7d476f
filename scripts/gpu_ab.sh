#!/bin/bash
# A/B of two builds of libpint_hip.so on the PTA bench leg (C2 leg too with C2=1):
# B = $LIB_B (default build/libpint_base.so, e.g. HEAD), A = the in-tree library.  Runs
# B, A, B, A and prints value / ms per step / kernel_ms of each; then the GPU parity tests
# of $1 (default none) on A.  Each GPU step has its own time limit; a failure ends the call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
LIB_B=${LIB_B:-build/libpint_base.so}
C2=${C2:-0}
for k in 1 2; do
  for v in B A; do
    if [ $v = B ]; then export PINT_LIB=$LIB_B; else unset PINT_LIB; fi
    timeout -k 10 240 python3 bench.py --grid 0 --j0740 0 --c2 $([ $C2 = 1 ] && echo 256 || echo 0) \
        --cpu-baseline 0 > gpurun_out/ab_$v$k.json 2> gpurun_out/ab_$v$k.err || { tail -5 gpurun_out/ab_$v$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v$k.json')); r=d['roofline']; print('$v$k', d['value'], d['ms_per_step'], {k: round(x, 4) for k, x in r['kernel_ms'].items()}, (d.get('c2') or {}).get('batched_fits_per_s'))"
  done
done
unset PINT_LIB
if [ -n "${1:-}" ]; then
  timeout -k 10 600 python -u -m pytest $1 -m gpu --maxfail=20 -q -rf -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_ab.log; exit $rc
fi
