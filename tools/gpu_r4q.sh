#!/bin/bash
# local forward (row groups in flight x waves per SIMD, k=64) and chunk backward (r1 rows in flight)
# build variants, same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4q
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
run() {  # preset tag variant
  FM_HIP_VARIANT=$3 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for rep in 1 2; do
  for V in base fu3w6 fu2w7 cu12 cu16; do
    T=$V; [ $V = base ] && V=""
    run k64 $T "$V" || exit 1
  done
done
for P in k64_bf16 k16_bf16 k128_fp8_ftrl; do
  for rep in 1 2; do
    for V in base cu12 cu16; do
      T=$V; [ $V = base ] && V=""
      run $P $T "$V" || exit 1
    done
  done
done
