# PMC instruction mix of the bench kernels (one rocprofv3 pass, SQ counters only)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 1 --warmup 0 --grid 0 --cpu-baseline 0 > gpurun_out/pmc_sq.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_sq.log; exit $rc
