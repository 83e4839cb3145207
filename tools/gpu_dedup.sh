#!/bin/bash
# Dedup chain cost on one box: tools/side_chain_cost.py (full step / compute chain / dedup chain) per
# sort algorithm and hot-row setting, then tools/bench_dedup.py (the dedup alone) with kernel profiles.
# usage: tools/gpu_dedup.sh <tag>
set -o pipefail
TAG=${1:-dedup}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for V in "FM_DEDUP_SORT=onesweep FM_HOT_ROWS=0" "FM_DEDUP_SORT=bucket FM_HOT_ROWS=0" "FM_DEDUP_SORT=onesweep FM_HOT_ROWS=1" "FM_DEDUP_SORT=bucket FM_HOT_ROWS=1"; do
  env $V timeout -k 10 240 python tools/side_chain_cost.py --steps 30 > $OUT/sc.log 2>&1 || { echo "side chain failed: $V"; tail -20 $OUT/sc.log; exit 1; }
  echo "[$V] $(grep side_chain $OUT/sc.log)"
done
timeout -k 10 200 python tools/bench_dedup.py > $OUT/bd.log 2>&1 || { echo "bench_dedup failed"; tail -20 $OUT/bd.log; exit 1; }
grep bench_dedup $OUT/bd.log
cd /tmp && export TMPDIR=/tmp
for V in onesweep bucket; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o run -- python3 $R/tools/bench_dedup.py --algo $V --iters 20 > $OUT/prof_$V.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$V.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof_$V/run_kernel_stats.csv 1 > $OUT/k_$V.txt
  rm -f $OUT/prof_$V/run_kernel_trace.csv
  echo "== $V"; grep -E "part_|bucket_sort|rle_|rocprim" $OUT/k_$V.txt | cut -c1-150
done
