#!/bin/bash
# Chunk-kernel grid cap (FM_CHUNK_GRID) sweep per preset, alternating.
set -o pipefail
TAG=${1:-grid_ab2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for PV in "k16_bf16 0 256 384 512 640" "k64 0 1536 2304 3072" "k64_bf16 0 512 768" "k128_fp8_ftrl 0 384 512 768" "k128_ftrl 0 512"; do
    set -- $PV; P=$1; shift
    for GC in "$@"; do
      FM_CHUNK_GRID=$GC timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$GC.json 2> $OUT/b_${P}_$GC.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$GC.err; exit 1; }
      echo "rep$rep $P chunk_grid=$GC: $(grep ms/step $OUT/b_${P}_$GC.err)"
    done
  done
done
