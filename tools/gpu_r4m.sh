#!/bin/bash
# per-kernel profile: row-sharded step at world 1 vs the local step (k64 fp32)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4m
mkdir -p $OUT
export FM_NO_AUTOBUILD=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
cd /tmp && export TMPDIR=/tmp
for M in shard local; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$M -o run -- python3 $R/bench.py --mode $M --gpus 1 --steps 30 --warmup 5 > $OUT/b_$M.json 2> $OUT/b_$M.err || { echo "prof $M failed"; tail -20 $OUT/b_$M.err; exit 1; }
  echo "$M: $(grep ms/step $OUT/b_$M.err)"
  python3 $R/tools/kstats.py $OUT/prof_$M 35 > $OUT/kstats_$M.txt || true
  find $OUT/prof_$M -type f -name "*kernel_trace.csv" -delete
done
