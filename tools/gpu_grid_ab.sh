#!/bin/bash
# Chunk-kernel grid cap (FM_CHUNK_GRID) A/B on the local step, alternating.
set -o pipefail
TAG=${1:-grid_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for P in k64 k16_bf16; do
    for GC in 0 1024 768 512; do
      FM_CHUNK_GRID=$GC timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$GC.json 2> $OUT/b_${P}_$GC.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$GC.err; exit 1; }
      echo "rep$rep $P chunk_grid=$GC: $(grep ms/step $OUT/b_${P}_$GC.err)"
    done
    FM_CHUNK_GRID=768 FM_CHUNK_PIPE=1 timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_p.json 2> $OUT/b_${P}_p.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_p.err; exit 1; }
    echo "rep$rep $P chunk_grid=768 pipe=1: $(grep ms/step $OUT/b_${P}_p.err)"
  done
done
