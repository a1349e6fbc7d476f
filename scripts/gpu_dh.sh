set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in head r4; do
  d=.; [ $t = r4 ] && d=ab_r4
  rm -rf gpurun_out/dh_$t
  (cd $d && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OLDPWD/gpurun_out/dh_$t -o run -- python3 scripts/diag/downhill_split.py > $OLDPWD/gpurun_out/dh_$t.txt 2>&1) || exit 1
  f=$(find gpurun_out/dh_$t -name "*kernel_trace.csv" | head -1)
  python3 scripts/diag/downhill_split.py --trace "$f" gpurun_out/dh_$t.txt > gpurun_out/dh_${t}_split.txt
done
cat gpurun_out/dh_*_split.txt
