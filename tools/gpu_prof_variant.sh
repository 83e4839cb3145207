#!/bin/bash
# Kernel profile + timeline of one bench variant.  usage: tools/gpu_prof_variant.sh <tag> <marker-kernel> [bench args]
set -o pipefail
TAG=${1:-pv}; MARK=${2:-fm_fwd_kernel}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
grep ms/step $OUT/prof.log
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary.txt
MC=$(ls $OUT/prof/*memory_copy_trace.csv 2>/dev/null | head -1)
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv $MARK $MC > $OUT/timeline.txt
rm -f $OUT/prof/*.csv  # (per-dispatch traces: keep the summaries, stay under gpurun's merge-back limit)
