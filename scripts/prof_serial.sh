# kernel-trace profile with side-stream kernels serialised (isolated per-kernel durations)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export PINT_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profs -o run -- python3 bench.py --steps 5 --warmup 1 --grid 0 --cpu-baseline 0 > gpurun_out/profs.log 2>&1
rc=$?; tail -2 gpurun_out/profs.log; exit $rc
