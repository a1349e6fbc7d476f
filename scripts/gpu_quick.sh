set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --grid 64 --cpu-baseline 0 > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
rc=$?; cat gpurun_out/bench_q.json; tail -3 gpurun_out/bench_q.err; exit $rc
