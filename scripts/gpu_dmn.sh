#!/bin/bash
# The phoff_dmn parity tests first (PLDMNoise + frozen PHOFF), then the whole GPU suite.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k phoff_dmn > gpurun_out/pytest_dmn.log 2>&1 || { tail -40 gpurun_out/pytest_dmn.log; exit 1; }
grep -c PASSED gpurun_out/pytest_dmn.log; grep -i "chi2 rel" gpurun_out/pytest_dmn.log | head
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
