#!/bin/bash
# Fused singleton update: its GPU tests, then an alternating same-box A/B (FM_FWD_SINGLE=0/1)
# over the bench presets (local and row-sharded world-1 steps) and kernel profiles.
# A numeric test failure is reported and the A/B still runs; a crash / timeout ends the script.
# usage: tools/gpu_single_ab.sh <tag>
set -o pipefail
TAG=${1:-single_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_fwd_single_gpu.py tests/test_step_gpu.py -v --timeout 120 --timeout-method thread > $OUT/pytest_single.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|differ" $OUT/pytest_single.log | tail -40
tail -1 $OUT/pytest_single.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for rep in 1 2; do
  for P in k64 k64_bf16 k16_bf16 k128_fp8_ftrl k128_ftrl; do
    for F in 0 1; do
      FM_FWD_SINGLE=$F timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$F.json 2> $OUT/b_${P}_$F.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$F.err; exit 1; }
      echo "rep$rep $P fwd_single=$F: $(grep ms/step $OUT/b_${P}_$F.err)"
    done
  done
  for F in 0 1; do
    FM_FWD_SINGLE=$F timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --prefetch-rows on --steps 40 --warmup 5 > $OUT/b_shard_$F.json 2> $OUT/b_shard_$F.err || { echo "shard bench failed"; tail -20 $OUT/b_shard_$F.err; exit 1; }
    echo "rep$rep shard(early rows on) fwd_single=$F: $(grep ms/step $OUT/b_shard_$F.err)"
  done
done
cd /tmp && export TMPDIR=/tmp
for F in 0 1; do
  FM_FWD_SINGLE=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$F -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $OUT/prof$F.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof$F.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof$F/run_kernel_stats.csv 25 > $OUT/kernel_summary_single$F.txt
  python3 $R/tools/timeline.py $OUT/prof$F/run_kernel_trace.csv fm_fwd > $OUT/timeline_single$F.txt
  head -8 $OUT/kernel_summary_single$F.txt
  rm -f $OUT/prof$F/run_kernel_trace.csv
done
exit $rc
