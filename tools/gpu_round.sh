#!/bin/bash
# Round check on the GPU box: GPU tests, smoke, default bench, row-sharded bench at world 1.
# usage: tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --steps 30 --warmup 5 > $OUT/bench_shard.json 2> $OUT/bench_shard.err || { echo "shard bench failed"; tail -20 $OUT/bench_shard.err; exit 1; }
echo "shard: $(grep ms/step $OUT/bench_shard.err)"
