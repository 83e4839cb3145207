#!/bin/bash
# Side-stream priority and lookahead depth re-checked with the chunk workgroup cap, alternating.
set -o pipefail
TAG=${1:-prio2_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for P in k64 k16_bf16; do
    for V in "0 1" "-1 1" "0 0"; do
      set -- $V
      FM_SIDE_PRIORITY=$1 FM_LOCAL_DEPTH2=$2 timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
      echo "rep$rep $P side_priority=$1 depth2=$2: $(grep ms/step $OUT/b.err)"
    done
  done
done
