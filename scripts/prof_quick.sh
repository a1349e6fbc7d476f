# kernel-trace profile of a short bench run (no PMC)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profq -o run -- python3 bench.py --steps 20 --warmup 2 --grid 0 --j0740 0 --cpu-baseline 0 > gpurun_out/profq.log 2>&1
rc=$?; tail -2 gpurun_out/profq.log; exit $rc
