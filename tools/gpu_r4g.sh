#!/bin/bash
# k16 bf16 / k128 bf16 FTRL regression bisect: head (c1da72d) vs h1 (c1da72d + the working tree's
# hdedup.hip / feeder.hip / module.hip) vs the working tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4g
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
run() {  # preset tag dir variant
  (cd $3 && FM_HIP_VARIANT=$4 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err) || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k16_bf16; do
  for rep in 1 2 3; do
    run $P head $R/ab/head "" || exit 1
    run $P h1 $R/ab/h1 "" || exit 1
    run $P h2fwd $R/ab/h2 "" || exit 1
    run $P h3bwd $R/ab/h3 "" || exit 1
    run $P new $R "" || exit 1
  done
done
