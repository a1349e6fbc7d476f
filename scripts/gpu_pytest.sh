#!/bin/bash
# pytest -m gpu on the box (selection in $1, default all), output to gpurun_out/pytest_<tag>.log
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SEL=${1:-tests}
TAG=${2:-sel}
timeout -k 10 900 python -u -m pytest $SEL -m gpu ${PYX:--x} -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|error|: " gpurun_out/pytest_$TAG.log | tail -60
exit $rc
