for V in "ROC_ACTIVE_WAIT_TIMEOUT=1000000" "ROC_ACTIVE_WAIT_TIMEOUT=0" "HIP_DUMMY=0"; do
for i in 1 2 3 4; do
  env $V timeout -k 10 120 python3 bench.py --steps 20 --grid 0 --j0740 0 --c2 0 --cpu-baseline 0 --emulate-world "" --cold-start 0 2> gpurun_out/tr$i.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$V steps20', d['ms_per_step'])" || exit 1
done
done
