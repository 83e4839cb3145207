#!/bin/bash
# Chunk-kernel workgroup cap in the row-sharded step (world 1, early rows on), alternating.
set -o pipefail
TAG=${1:-sgrid_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2 3; do
  for GC in -1 0 2304 4608; do
    FM_CHUNK_GRID=$GC timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --prefetch-rows on --steps 40 --warmup 5 > $OUT/b_$GC.json 2> $OUT/b_$GC.err || { echo "shard bench failed"; tail -20 $OUT/b_$GC.err; exit 1; }
    echo "rep$rep shard chunk_grid=$GC: $(grep ms/step $OUT/b_$GC.err)"
  done
done
