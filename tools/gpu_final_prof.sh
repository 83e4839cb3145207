#!/bin/bash
# Kernel profile (rocprofv3 --kernel-trace --stats) of the default bench step: summary + one-step timeline.
set -o pipefail
TAG=${1:-final_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary.txt
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline.txt
head -12 $OUT/kernel_summary.txt | cut -c1-130
head -3 $OUT/timeline.txt
rm -f $OUT/prof/run_kernel_trace.csv
