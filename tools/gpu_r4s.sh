#!/bin/bash
# local forward of 32-lane rows (k=128): fp8 UNR4/W7 (default) vs UNR12/W4 control, bf16 unchanged
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4s
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
run() {  # preset tag variant
  FM_HIP_VARIANT=$3 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k128_fp8_ftrl k128_ftrl; do
  for rep in 1 2; do
    for V in base f8u12w4; do
      T=$V; [ $V = base ] && V=""
      run $P $T "$V" || exit 1
    done
  done
done
