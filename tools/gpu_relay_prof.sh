#!/bin/bash
# Kernel profile of the row-sharded step at world 2 on one GPU (tools/relay_bench.py, host relay).
set -o pipefail
TAG=${1:-relay_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/tools/relay_bench.py --world 2 --steps 8 > $OUT/relay.log 2>&1 || { echo "relay bench failed"; tail -30 $OUT/relay.log; exit 1; }
grep relay_bench $OUT/relay.log
find $OUT/prof -name "*kernel_stats.csv" | head
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do python3 $R/tools/kstats.py $f 22 | head -28; done > $OUT/kstats_relay.txt
cat $OUT/kstats_relay.txt | cut -c1-150
find $OUT/prof -name "*kernel_trace.csv" -delete
