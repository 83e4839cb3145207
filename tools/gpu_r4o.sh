#!/bin/bash
# sharded k128 fp8 FTRL at world 1 under the exchange options (early rows, split grads, self rows)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4o
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for V in "on on 1" "on off 1" "off off 1" "on off 0" "on on 1"; do
  set -- $V
  T=fp8_$1_$2_self$3
  FM_SELF_ROWS=$3 timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 1 --preset k128_fp8_ftrl --mode shard --prefetch-rows $1 --overlap-grads $2 --steps 30 --warmup 5 > $OUT/$T.json 2> $OUT/$T.err || { echo "shard $T failed"; tail -20 $OUT/$T.err; exit 1; }
  echo "shard fp8 (early rows $1, split grads $2, self rows $3): $(grep ms/step $OUT/$T.err)"
done
