#!/bin/bash
# per-kernel time of the EMIT path (world > 1 compute proxy) vs the local step, k128 fp8 FTRL
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4x
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29641
for M in local shard; do
  export MASTER_PORT=$((MASTER_PORT+1)) FM_SHARD_W1_LOCAL=0
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$M -- python3 $R/bench.py --gpus 1 --preset k128_fp8_ftrl --mode $M --steps 40 --warmup 5 > $OUT/p_$M.json 2> $OUT/p_$M.err || { echo "prof $M failed"; tail -20 $OUT/p_$M.err; exit 1; }
  find $OUT/prof_$M -name '*kernel_trace.csv' -delete
  echo "== $M: $(grep ms/step $OUT/p_$M.err)"
  python3 $R/tools/kstats.py $OUT/prof_$M 45 | grep -v "at::native::\(vectorized\|elementwise\|distribution\|(anonymous\)" 
done
