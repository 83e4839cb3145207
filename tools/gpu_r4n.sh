#!/bin/bash
# sharded k128 fp8 FTRL at world 1: ab/head (c5df060, before the fp8 row norms) vs the working tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4n
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
shard() {  # tag dir
  (cd $2 && timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 1 --preset k128_fp8_ftrl --mode shard --steps 30 --warmup 5 > $OUT/shard_$1.json 2> $OUT/shard_$1.err) || { echo "shard $1 failed"; tail -20 $OUT/shard_$1.err; return 1; }
  echo "shard fp8 $1: $(grep ms/step $OUT/shard_$1.err)"
}
for rep in 1 2; do shard head $R/ab/head || exit 1; shard new $R || exit 1; done
