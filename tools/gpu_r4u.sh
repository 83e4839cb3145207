#!/bin/bash
# kernel timeline of one step: local vs sharded (world 1) k64 fp32
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4u
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
for M in shard; do
  export MASTER_PORT=$((MASTER_PORT+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$M -- python3 $R/bench.py --gpus 1 --mode $M --steps 20 --warmup 5 > $OUT/t_$M.json 2> $OUT/t_$M.err || { echo "trace $M failed"; tail -20 $OUT/t_$M.err; exit 1; }
  F=$(find $OUT/tr_$M -name '*kernel_trace.csv' | head -1)
  MK=fm_fwd_kernel
  python3 $R/tools/timeline.py $F $MK > $OUT/timeline_$M.txt
  rm -f $F
  echo "== $M: $(grep ms/step $OUT/t_$M.err)"
  cat $OUT/timeline_$M.txt
done
