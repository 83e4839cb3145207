#!/bin/bash
# Chunk-kernel grid cap (FM_CHUNK_GRID) sweep around the optima, alternating.
set -o pipefail
TAG=${1:-grid_ab3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for PV in "k64 0 2688 3072 3456 3840 4608 6144" "k64_bf16 0 3072 3840" "k16_bf16 0 512 576"; do
    set -- $PV; P=$1; shift
    for GC in "$@"; do
      FM_CHUNK_GRID=$GC timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$GC.json 2> $OUT/b_${P}_$GC.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$GC.err; exit 1; }
      echo "rep$rep $P chunk_grid=$GC: $(grep ms/step $OUT/b_${P}_$GC.err)"
    done
  done
done
