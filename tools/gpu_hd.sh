#!/bin/bash
# Hot-dictionary dedup check: its GPU tests, the dedup chain alone (hd vs onesweep), a kernel
# profile of the hd chain, and the step A/B.  usage: tools/gpu_hd.sh <tag>
set -o pipefail
TAG=${1:-hd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hd_dedup_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_hd.log 2>&1 || { echo "hd tests failed"; tail -40 $OUT/pytest_hd.log; exit 1; }
tail -3 $OUT/pytest_hd.log
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu_relay.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_relay.log 2>&1
rc=$?
tail -5 $OUT/pytest_relay.log
case $rc in 0|1) ;; *) echo "relay tests rc=$rc: stopping"; exit 1;; esac
timeout -k 10 200 python tools/bench_dedup.py --algo onesweep,hd > $OUT/bench_dedup.txt 2>&1 || { echo "bench_dedup failed"; tail -20 $OUT/bench_dedup.txt; exit 1; }
cat $OUT/bench_dedup.txt
for V in onesweep hd onesweep hd; do
  FM_DEDUP=$V timeout -k 10 200 python bench.py --steps 40 --warmup 8 > $OUT/bench_$V.json 2> $OUT/bench_$V.err || { echo "bench $V failed"; tail -20 $OUT/bench_$V.err; exit 1; }
  echo "FM_DEDUP=$V: $(grep ms/step $OUT/bench_$V.err)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_dedup -o run -- python3 $R/tools/bench_dedup.py --algo hd --iters 10 > $OUT/prof_dedup.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_dedup.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof_dedup/run_kernel_stats.csv 40 > $OUT/kernel_summary_dedup.txt
cat $OUT/kernel_summary_dedup.txt | head -45
rm -f $OUT/prof_dedup/run_kernel_trace.csv
timeout -k 10 60 rocprofv3 --list-avail > $OUT/counters_avail.txt 2>&1 || echo "list-avail rc=$?"
grep -c . $OUT/counters_avail.txt
