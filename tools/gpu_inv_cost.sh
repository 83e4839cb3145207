#!/bin/bash
# Price of the sharded dedup's inverse-map scatter (tools/inv_cost.py), alternating, + kernel stats.
set -o pipefail
TAG=${1:-inv_cost}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for I in 0 1; do
    timeout -k 10 200 python tools/inv_cost.py --inv $I > $OUT/inv$I.log 2>&1 || { echo "inv_cost $I failed"; tail -20 $OUT/inv$I.log; exit 1; }
    grep inv_cost $OUT/inv$I.log
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/tools/inv_cost.py --inv 1 --steps 20 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kstats_inv1.txt
grep -h "rle_tile\|fm_fwd\|chunk" $OUT/kstats_inv1.txt
rm -f $OUT/prof/run_kernel_trace.csv
