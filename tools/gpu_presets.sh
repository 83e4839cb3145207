#!/bin/bash
# All bench presets + the row-sharded path at world 1 (RCCL), then a kernel profile of the sharded step.
# usage: tools/gpu_presets.sh <tag>
set -o pipefail
TAG=${1:-presets}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for P in k64 k64_bf16 k16_bf16 k128_ftrl k128_fp8_ftrl k64_dp_dense; do
  timeout -k 10 300 python bench.py --preset $P --steps 30 --warmup 5 > $OUT/bench_$P.json 2> $OUT/bench_$P.err || { echo "bench $P failed"; tail -20 $OUT/bench_$P.err; exit 1; }
  echo "$P: $(tail -1 $OUT/bench_$P.err)"
done
# sharded step at world 1: (early rows, split grads, self rows); "on off 1" = the N>1 defaults
for V in "off off 1" "on off 1" "on on 1" "on off 0"; do
  set -- $V
  T=shard_$1_$2_self$3
  FM_SELF_ROWS=$3 timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --prefetch-rows $1 --overlap-grads $2 --steps 30 --warmup 5 > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { echo "shard bench failed"; tail -20 $OUT/bench_$T.err; exit 1; }
  echo "shard (early rows $1, split grads $2, self rows $3): $(grep ms/step $OUT/bench_$T.err)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard -o run -- python3 $R/bench.py --mode shard --prefetch-rows on --steps 20 --warmup 5 > $OUT/prof_shard.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_shard.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof_shard/run_kernel_stats.csv 30 > $OUT/kernel_summary_shard.txt
python3 $R/tools/timeline.py $OUT/prof_shard/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline_shard.txt
rm -f $OUT/prof_shard/run_kernel_trace.csv
