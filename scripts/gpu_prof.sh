#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel stats of the bench workload (PTA; C2; the
# NGC6440E grid alone), the HBM PMC passes (FETCH_SIZE, WRITE_SIZE: one counter group per
# run) of the PTA and of the grid, the Gram MFMA / LDS / activity passes and the grid's VALU
# pass.  Outputs under gpurun_out/; summaries are made on the host by scripts/*_summary.py.
# Each GPU step has its own time limit; any failure stops it.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export PINT_GRID_PIPES=1  # (per-kernel figures of one session: no concurrent grid blocks)
# the 68-pulsar PTA step only: no emulated shards, no cold start (their launches would mix
# other batch sizes into the per-kernel figures)
B="python3 bench.py --steps 2 --warmup 1 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 --pipes 1"
# kernel stats at the bench's own length (100 timed steps, steady clocks), its line beside
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 100 --warmup 10 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 --pipes 1 \
    > gpurun_out/prof.json 2> gpurun_out/prof.log || exit $?
# C2 (B1855 x 256 batched fits) on its own trace: its kernels share names with the PTA's
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- \
    python3 bench.py --steps 2 --warmup 1 --npsr 4 --grid 0 --j0740 0 --cpu-baseline 0 --emulate-world 0 --cold-start 0 --pipes 1 \
    > gpurun_out/prof_c2.log 2>&1 || exit $?
# the (F0, F1) grid alone
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_grid -o run -- \
    python3 scripts/grid_run.py 256 > gpurun_out/prof_grid.json 2> gpurun_out/prof_grid.log || exit $?
G="python3 scripts/grid_run.py 256"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcg_fetch -o run -- $G > gpurun_out/pmcg_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcg_write -o run -- $G > gpurun_out/pmcg_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcg_valu -o run -- $G > gpurun_out/pmcg_valu.log 2>&1 || exit $?
export PINT_SERIAL=1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma -o run -- $B > gpurun_out/pmc_mfma.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_lds -o run -- $B > gpurun_out/pmc_lds.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_act -o run -- $B > gpurun_out/pmc_act.log 2>&1 || exit $?
echo prof-done
