#!/bin/bash
# A/B: side-stream priority (FM_SIDE_PRIORITY 0 vs -1), local and sharded step, alternating runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prio}
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for P in 0 -1; do
    for M in local shard; do
      FM_SIDE_PRIORITY=$P timeout -k 10 300 python bench.py --mode $M --steps 50 --warmup 10 > $OUT/b_${M}_${P}_$rep.json 2> $OUT/b_${M}_${P}_$rep.err || { echo "bench failed"; tail -20 $OUT/b_${M}_${P}_$rep.err; exit 1; }
      echo "prio=$P mode=$M rep=$rep: $(grep ms/step $OUT/b_${M}_${P}_$rep.err)"
    done
  done
done
