# PMC passes on the bench for the Gram stage: MFMA busy / instruction counts and LDS
# behaviour (one pass per counter group, each its own run)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export PINT_SERIAL=1
run() {  # run <name> <counters...>
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o run -- python3 bench.py --steps 1 --warmup 0 --grid 0 --j0740 0 --cpu-baseline 0 > gpurun_out/pmc_$name.log 2>&1
}
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit $?
run lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS || exit $?
run act SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VALU || exit $?
