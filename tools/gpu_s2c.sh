#!/bin/bash
# Dedup chain alone: wall time per algorithm, then per-kernel profiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r3s2c
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
timeout -k 10 200 python tools/bench_dedup.py > $OUT/bd.log 2>&1 || { echo "bench_dedup failed"; tail -20 $OUT/bd.log; exit 1; }
grep bench_dedup $OUT/bd.log
cd /tmp && export TMPDIR=/tmp
for V in onesweep bucket; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o run -- python3 $R/tools/bench_dedup.py --algo $V --iters 20 > $OUT/prof_$V.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$V.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof_$V/run_kernel_stats.csv 1 > $OUT/k_$V.txt
  rm -f $OUT/prof_$V/run_kernel_trace.csv
  echo "== $V"; grep -E "part_|bucket_sort|rle_|rocprim|fill|copy" $OUT/k_$V.txt | cut -c1-150
done
