set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "grid" > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_j.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --grid 64 --j0740 ${J0740:-16} --cpu-baseline 0 > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err
rc=$?; cat gpurun_out/bench_j.json; tail -5 gpurun_out/bench_j.err; exit $rc
