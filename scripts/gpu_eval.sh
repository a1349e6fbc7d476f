#!/bin/bash
# Evaluation-kernel diagnosis: block phase split at 68 and 9 pulsars, one SQ PMC pass of the
# PTA step (instruction mix, wave cycles, waits).  Each GPU step has its own time limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/diag/eval_phases.py 68 5 > gpurun_out/evp68.txt 2>&1 || { tail -20 gpurun_out/evp68.txt; exit 1; }
cat gpurun_out/evp68.txt
timeout -k 10 200 python3 scripts/diag/eval_phases.py 9 5 > gpurun_out/evp9.txt 2>&1 || { tail -20 gpurun_out/evp9.txt; exit 1; }
cat gpurun_out/evp9.txt
rm -rf gpurun_out/pmc_ev
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d gpurun_out/pmc_ev -o run -- python3 bench.py --steps 2 --warmup 1 --grid 0 --j0740 0 --c2 0 \
    --cpu-baseline 0 --emulate-world 0 --cold-start 0 > gpurun_out/pmc_ev.log 2>&1 || { tail -5 gpurun_out/pmc_ev.log; exit 1; }
f=$(find gpurun_out/pmc_ev -name "*counter_collection.csv" | head -1); python3 scripts/pmc_table.py "$(dirname "$f")" > gpurun_out/pmc_ev.txt 2>&1; cat gpurun_out/pmc_ev.txt
