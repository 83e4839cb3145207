#!/bin/bash
# Segment lookup (FM_SEG_LOOKUP) in the row-sharded step: GPU tests, then alternating A/B of the
# world-1 sharded bench (early rows on = the N>1 default; off) and a kernel profile.
# usage: tools/gpu_seg_ab.sh <tag>
set -o pipefail
TAG=${1:-seg_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_seg.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest_seg.log | head -30; tail -30 $OUT/pytest_seg.log; exit 1; }
tail -1 $OUT/pytest_seg.log
for rep in 1 2 3; do
  for PF in on off; do
    for F in 0 1; do
      FM_SEG_LOOKUP=$F timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --prefetch-rows $PF --steps 40 --warmup 5 > $OUT/b_$PF$F.json 2> $OUT/b_$PF$F.err || { echo "shard bench failed"; tail -20 $OUT/b_$PF$F.err; exit 1; }
      echo "rep$rep shard early_rows=$PF seg_lookup=$F: $(grep ms/step $OUT/b_$PF$F.err)"
    done
  done
done
for P in k128_fp8_ftrl k16_bf16; do
  for F in 0 1; do
    FM_SEG_LOOKUP=$F timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --preset $P --mode shard --prefetch-rows on --steps 40 --warmup 5 > $OUT/b_$P$F.json 2> $OUT/b_$P$F.err || { echo "shard bench failed"; tail -20 $OUT/b_$P$F.err; exit 1; }
    echo "shard $P early_rows=on seg_lookup=$F: $(grep ms/step $OUT/b_$P$F.err)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --mode shard --prefetch-rows on --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary_shard_seg.txt
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline_shard_seg.txt
head -14 $OUT/kernel_summary_shard_seg.txt
rm -f $OUT/prof/run_kernel_trace.csv
