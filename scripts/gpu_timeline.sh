#!/bin/bash
# One steady step's kernel timeline (rocprofv3 kernel trace -> scripts/step_timeline.py) of the
# PTA step at NPSR pulsars (default 9: the per-rank shard of the 8-GPU headline), plus the
# k_solve_dmx phase stamps of workgroup 0 (scripts/diag/ts_probe.py).  One pipeline (PIPES=2: two
# sessions fed round-robin, their steps interleaved in the trace).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-9}
rm -rf gpurun_out/tl$N
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl$N -o run -- \
    python3 bench.py --npsr $N --steps 60 --warmup 10 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world "" \
    --cold-start 0 --pipes ${PIPES:-1} > gpurun_out/tl$N.json 2> gpurun_out/tl$N.err || { tail -5 gpurun_out/tl$N.err; exit 1; }
f=$(find gpurun_out/tl$N -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$f" > gpurun_out/timeline_$N.txt
cat gpurun_out/timeline_$N.txt
timeout -k 10 120 python3 scripts/diag/ts_probe.py $N apply > gpurun_out/ts$N.txt 2>&1 || { tail -5 gpurun_out/ts$N.txt; exit 1; }
cat gpurun_out/ts$N.txt
