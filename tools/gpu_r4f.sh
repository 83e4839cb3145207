#!/bin/bash
# k16 bf16 regression hunt: committed tree (ab/head) vs working tree vs its allgen variant (HEAD's
# forward / chunk-kernel ISA), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4f
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
run() {  # preset tag dir variant
  (cd $3 && FM_HIP_VARIANT=$4 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err) || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k16_bf16 k128_ftrl k64; do
  for rep in 1 2 3; do
    run $P head $R/ab/head "" || exit 1
    run $P new $R "" || exit 1
    run $P allgen $R allgen || exit 1
  done
done
