#!/bin/bash
# Dist GPU tests, then sharded-step benches (world 1, RCCL) for wire-format variants.
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
  timeout -k 10 300 python bench.py --mode shard --steps 30 --warmup 5 "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; exit 1; }
  echo "$n: $(grep ms/step $OUT/$n.err)"
}
run shard_fp32
run shard_bf16wire --comm-dtype bf16
run shard_k16bf16 --preset k16_bf16
run shard_k128fp8 --preset k128_fp8_ftrl
timeout -k 10 300 python bench.py --preset k16_bf16 --steps 30 --warmup 5 > $OUT/local_k16bf16.json 2> $OUT/local_k16bf16.err && echo "local_k16bf16: $(grep ms/step $OUT/local_k16bf16.err)"
timeout -k 10 300 python bench.py --preset k128_fp8_ftrl --steps 30 --warmup 5 > $OUT/local_k128fp8.json 2> $OUT/local_k128fp8.err && echo "local_k128fp8: $(grep ms/step $OUT/local_k128fp8.err)"
