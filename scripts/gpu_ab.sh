#!/bin/bash
# Single-fit legs A/B: HEAD (system HIP runtime, then torch's) against an older tree checked
# out at ab_r4/ (git worktree, library built in place), scripts/diag/ab_single.py in each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 240 python3 scripts/diag/ab_single.py --prof > gpurun_out/ab_head.txt 2>&1 || exit $?
PINT_HIP_RUNTIME=torch timeout -k 10 240 python3 scripts/diag/ab_single.py > gpurun_out/ab_head_torch.txt 2>&1 || exit $?
AB_ROOT=$PWD/ab_r4 timeout -k 10 240 python3 scripts/diag/ab_single.py --prof > gpurun_out/ab_r4.txt 2>&1 || exit $?
grep -h "ms:" gpurun_out/ab_*.txt
bash scripts/gpu_timeline.sh 9 > gpurun_out/tl9_out.txt 2>&1 || exit $?
