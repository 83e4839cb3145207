#!/bin/bash
# Row-sharded step at world 1 (RCCL): split-gradient backward on / off, alternating, one box.
# usage: tools/gpu_shard_ab.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-shard_ab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
i=0
for V in off on off on off on; do
  i=$((i+1))
  timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$i bench.py --gpus 1 --mode shard --prefetch-rows on --overlap-grads $V --steps 40 --warmup 5 "$@" > $OUT/v$i.json 2> $OUT/v$i.err || { echo "shard bench failed"; tail -20 $OUT/v$i.err; exit 1; }
  echo "[split grads $V $*] $(grep ms/step $OUT/v$i.err)"
done
