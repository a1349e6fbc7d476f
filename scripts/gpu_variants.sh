#!/bin/bash
# Bench several builds of libpint_hip.so on the PTA leg, interleaved (two rounds):
#   scripts/gpu_variants.sh "build/libpint_base.so build/libpint_x.so tree tree@PINT_EVAL_WPE=5" ["pytest selection" [lib]]
# "tree" is the in-tree library; "lib@VAR=value" runs that library with one environment setting.  Prints value / ms per step / kernel_ms per run; then, if a
# selection is given, runs it on $3 (default the in-tree library).  Each GPU step has its own
# time limit and a failure ends the call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
LIBS=$1
for k in 1 2; do
  for item in $LIBS; do
    lib=${item%%@*}; envset=""; [ "$item" != "$lib" ] && envset=${item#*@}
    tag=$(basename $lib .so)${envset:+_${envset//=/}}
    if [ $lib = tree ]; then unset PINT_LIB; else export PINT_LIB=$lib; fi
    env $envset timeout -k 10 240 python3 bench.py --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 \
        > gpurun_out/var_$tag$k.json 2> gpurun_out/var_$tag$k.err || { tail -5 gpurun_out/var_$tag$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/var_$tag$k.json')); r=d['roofline']; print('$tag$k', d['value'], d['ms_per_step'], {k: round(x, 4) for k, x in r['kernel_ms'].items()})"
  done
done
unset PINT_LIB
if [ -n "${2:-}" ]; then
  if [ -n "${3:-}" ] && [ "${3}" != tree ]; then export PINT_LIB=$3; fi
  timeout -k 10 600 python -u -m pytest $2 -m gpu --maxfail=20 -q -rf -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_var.log 2>&1
  rc=$?; tail -6 gpurun_out/pytest_var.log; exit $rc
fi
