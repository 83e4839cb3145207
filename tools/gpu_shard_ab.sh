#!/bin/bash
# Dist GPU tests, then sharded-step benches (world 1, RCCL) for variants.
# usage: tools/gpu_shard_ab.sh <tag>
set -o pipefail
TAG=${1:-shardab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; exit 1; }
  echo "$n: $(grep ms/step $OUT/$n.err)"
}
run shard_mb1 --mode shard
run shard_mb2 --mode shard --microbatches 2
run shard_mb1b --mode shard
run shard_mb2b --mode shard --microbatches 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --mode shard --microbatches 2 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary.txt
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv gather_ > $OUT/timeline.txt
cat $OUT/timeline.txt
