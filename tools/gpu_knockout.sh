#!/bin/bash
# Hot-row knockout (tools/knockout_hot.py) under a kernel trace, plus an alternating A/B of
# the dense-row MFMA backward (FM_DENSE_BWD) on the k=128 FTRL presets.
# usage: tools/gpu_knockout.sh <tag>
set -o pipefail
TAG=${1:-knockout}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for D in 0 64 256 1024; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ko$D -o run -- python3 $R/tools/knockout_hot.py --drop $D --steps 30 > $OUT/ko$D.log 2>&1 || { echo "knockout $D failed"; tail -30 $OUT/ko$D.log; exit 1; }
  grep knockout $OUT/ko$D.log
  python3 $R/tools/kstats.py $OUT/ko$D/run_kernel_stats.csv 35 > $OUT/kstats_ko$D.txt
  head -6 $OUT/kstats_ko$D.txt
  rm -f $OUT/ko$D/run_kernel_trace.csv
done
cd $R
for rep in 1 2; do
  for P in k128_fp8_ftrl k128_ftrl k64; do
    for DB in 0 1; do
      FM_DENSE_BWD=$DB timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$DB.json 2> $OUT/b_${P}_$DB.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$DB.err; exit 1; }
      echo "rep$rep $P dense_bwd=$DB: $(grep ms/step $OUT/b_${P}_$DB.err)"
    done
  done
done
