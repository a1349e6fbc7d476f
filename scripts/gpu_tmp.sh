timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --grid 256 --j0740 0 --c2 0 --cpu-baseline 0 2> gpurun_out/cold.err > gpurun_out/cold.json || exit 1
python3 scripts/bench_brief.py gpurun_out/cold.json
