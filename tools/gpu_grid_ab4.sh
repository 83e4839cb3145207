#!/bin/bash
# Chunk-kernel workgroup count above the old 8192 cap for 32-lane rows (k=128), alternating.
set -o pipefail
TAG=${1:-grid_ab4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for PV in "k128_fp8_ftrl 0 6144 12288 16384" "k128_ftrl 0 12288 16384"; do
    set -- $PV; P=$1; shift
    for GC in "$@"; do
      FM_CHUNK_GRID=$GC timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$GC.json 2> $OUT/b_${P}_$GC.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$GC.err; exit 1; }
      echo "rep$rep $P chunk_grid=$GC: $(grep ms/step $OUT/b_${P}_$GC.err)"
    done
  done
done
