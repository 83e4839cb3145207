#!/bin/bash
# Dedup chain cost: side_chain_cost for onesweep / bucket x hot rows off / on; dedup-only kernel profiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r3s2b
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
for V in "FM_DEDUP_SORT=onesweep FM_HOT_ROWS=0" "FM_DEDUP_SORT=bucket FM_HOT_ROWS=0" "FM_DEDUP_SORT=onesweep FM_HOT_ROWS=1" "FM_DEDUP_SORT=bucket FM_HOT_ROWS=1"; do
  env $V timeout -k 10 240 python tools/side_chain_cost.py --steps 30 > $OUT/sc.log 2>&1 || { echo "side chain failed: $V"; tail -20 $OUT/sc.log; exit 1; }
  echo "[$V] $(grep side_chain $OUT/sc.log)"
done
cd /tmp && export TMPDIR=/tmp
for V in onesweep bucket; do
  FM_DEDUP_SORT=$V FM_HOT_ROWS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o run -- python3 $R/tools/side_chain_cost.py --steps 20 --only dedup > $OUT/prof_$V.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$V.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof_$V/run_kernel_stats.csv 20 > $OUT/dedup_only_$V.txt
  rm -f $OUT/prof_$V/run_kernel_trace.csv
  echo "== dedup-only kernels ($V, hot rows), per step:"; grep -E "part_|bucket_sort|rle_|hot_|rocprim|csr_rows" $OUT/dedup_only_$V.txt | cut -c1-150
done
