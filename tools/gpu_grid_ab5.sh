#!/bin/bash
# Chunk-kernel workgroup cap on the dp_dense executor (EMIT_TABLE backward), alternating.
set -o pipefail
TAG=${1:-grid_ab5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for GC in 0 3840 2304; do
    FM_CHUNK_GRID=$GC timeout -k 10 200 python bench.py --preset k64_dp_dense --steps 40 --warmup 5 > $OUT/b_$GC.json 2> $OUT/b_$GC.err || { echo "bench failed"; tail -20 $OUT/b_$GC.err; exit 1; }
    echo "rep$rep k64_dp_dense chunk_grid=$GC: $(grep ms/step $OUT/b_$GC.err)"
  done
done
