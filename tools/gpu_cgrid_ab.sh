#!/bin/bash
# Combine / big-row kernel workgroup counts (FM_COMBINE_GRID, FM_BIG_GRID), alternating.
set -o pipefail
TAG=${1:-cgrid_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for V in "0 0" "512 0" "1024 0" "0 256" "0 512" "1024 512"; do
    set -- $V
    FM_COMBINE_GRID=$1 FM_BIG_GRID=$2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
    echo "rep$rep k64 combine_grid=$1 big_grid=$2: $(grep ms/step $OUT/b.err)"
  done
done
