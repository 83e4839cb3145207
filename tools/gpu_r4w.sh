#!/bin/bash
# EMIT-mode (world > 1) compute proxy: the sharded step at world 1 with FM_SHARD_W1_LOCAL=0,
# chunk workgroups per CU / chunk grid cap, alternating on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4w
mkdir -p $OUT
export FM_NO_AUTOBUILD=1 FM_SHARD_W1_LOCAL=0
cd $R
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
i=0
for P in "" "--preset k16_bf16" "--preset k128_fp8_ftrl"; do
  for rep in 1 2; do
    for V in "-1 0" "3 0" "3 3072" "2 0"; do
      set -- $V
      i=$((i+1)); export MASTER_PORT=$((29600+i))
      FM_CHUNK_WG_PER_CU=$1 FM_CHUNK_GRID=$2 timeout -k 10 300 python bench.py --gpus 1 --mode shard $P --steps 40 --warmup 8 > $OUT/v$i.json 2> $OUT/v$i.err || { echo "shard bench failed"; tail -20 $OUT/v$i.err; exit 1; }
      echo "[shard $P wg/cu=$1 grid=$2] $(grep ms/step $OUT/v$i.err)"
    done
  done
done
