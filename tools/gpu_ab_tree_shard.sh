#!/bin/bash
# Same-box A/B of the row-sharded step (world 1, default path) and the local step: this tree (with env
# variants) vs ab_old/ (see tools/gpu_ab_tree.sh for building ab_old/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abs
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
i=0
for args in "--mode shard" ""; do
  for side in "new" "new FM_BIG_BLOCKS=256" "new FM_BIG_BLOCKS=512" "new FM_BIG_BLOCKS=256" "new FM_BIG_BLOCKS=512" "new"; do
    i=$((i+1))
    if [ "$side" = old ]; then D=$R/ab_old; E=""; else D=$R; E=${side#new}; fi
    (cd $D && env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 $args > $OUT/r$i.json 2> $OUT/r$i.err) || { echo "run $i failed"; tail -20 $OUT/r$i.err; exit 1; }
    echo "[$side $args] $(grep ms/step $OUT/r$i.err)"
  done
done
