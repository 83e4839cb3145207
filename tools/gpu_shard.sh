#!/bin/bash
# GPU tests, then the row-sharded step at world 1 (RCCL): bench + kernel profile.
# usage: tools/gpu_shard.sh <tag>
set -o pipefail
TAG=${1:-shard}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --steps 30 --warmup 5 > $OUT/bench_shard.json 2> $OUT/bench_shard.err || { echo "shard bench failed"; tail -20 $OUT/bench_shard.err; exit 1; }
echo "shard: $(grep ms/step $OUT/bench_shard.err)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard -o run -- python3 $R/bench.py --mode shard --steps 20 --warmup 5 > $OUT/prof_shard.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_shard.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof_shard/run_kernel_stats.csv 30 > $OUT/kernel_summary_shard.txt
python3 $R/tools/timeline.py $OUT/prof_shard/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline_shard.txt
head -30 $OUT/kernel_summary_shard.txt
