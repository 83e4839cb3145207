#!/bin/bash
# Depth-2 lookahead of the local step (FM_LOCAL_DEPTH2) x pipelined chunk kernel (FM_CHUNK_PIPE):
# GPU step tests, then an alternating same-box A/B over the presets and a timeline.
# usage: tools/gpu_depth2_ab.sh <tag>
set -o pipefail
TAG=${1:-depth2_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_fwd_single_gpu.py tests/test_teardown_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_d2.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest_d2.log | head -30; tail -30 $OUT/pytest_d2.log; exit 1; }
tail -1 $OUT/pytest_d2.log
for rep in 1 2; do
  for P in k64 k64_bf16 k16_bf16 k128_fp8_ftrl; do
    for V in "0 0" "1 0" "1 1"; do
      set -- $V
      FM_LOCAL_DEPTH2=$1 FM_CHUNK_PIPE=$2 timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$1$2.json 2> $OUT/b_${P}_$1$2.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$1$2.err; exit 1; }
      echo "rep$rep $P depth2=$1 pipe=$2: $(grep ms/step $OUT/b_${P}_$1$2.err)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
FM_LOCAL_DEPTH2=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary_d2.txt
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline_d2.txt
head -3 $OUT/timeline_d2.txt
rm -f $OUT/prof/run_kernel_trace.csv
