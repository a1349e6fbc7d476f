#!/bin/bash
# 9-pulsar step timelines under a list of environment settings (one rocprof kernel trace each):
#   bash scripts/gpu_sweep.sh VAR "v1 v2 ..." [NPSR]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=$1; VALS=$2; N=${3:-9}
for v in $VALS; do
  d=gpurun_out/sw_${VAR}_$v
  rm -rf $d
  env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --npsr $N --steps 60 --warmup 10 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world "" \
    --cold-start 0 > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "== $VAR=$v"
  python3 scripts/step_timeline.py "$f" | head -22
done
