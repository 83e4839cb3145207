#!/bin/bash
# sharded step at world 1 vs the local step (k64 fp32): per-kernel time of both, and the
# split-gradient / early-row options at world 1 for k64 and k128 fp8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4t
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
for M in local shard; do
  export MASTER_PORT=$((MASTER_PORT+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$M -- python3 $R/bench.py --gpus 1 --mode $M --steps 40 --warmup 5 > $OUT/p_$M.json 2> $OUT/p_$M.err || { echo "prof $M failed"; tail -20 $OUT/p_$M.err; exit 1; }
  find $OUT/prof_$M -name '*kernel_trace.csv' -delete
  echo "== $M: $(grep ms/step $OUT/p_$M.err)"
  python3 $R/tools/kstats.py $OUT/prof_$M 45
done
cd $R
i=0
for P in "" "--preset k128_fp8_ftrl"; do
  for V in "--prefetch-rows auto --overlap-grads on" "--prefetch-rows auto --overlap-grads off" "--prefetch-rows on --overlap-grads off"; do
    i=$((i+1)); export MASTER_PORT=$((29550+i))
    timeout -k 10 300 python bench.py --gpus 1 --mode shard $P $V --steps 40 --warmup 8 > $OUT/v$i.json 2> $OUT/v$i.err || { echo "shard bench failed"; tail -20 $OUT/v$i.err; exit 1; }
    echo "[shard $P $V] $(grep ms/step $OUT/v$i.err)"
  done
done
