#!/bin/bash
# local forward of 4-lane rows (k=16 bf16): row groups in flight x waves per SIMD, same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4z
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for V in base f4u5w4 f4u6w4 f4u8w3 f4u4w5; do
    T=$V; [ $V = base ] && V=""
    FM_HIP_VARIANT=$V timeout -k 10 200 python bench.py --preset k16_bf16 --steps 40 --warmup 8 > $OUT/b_$T_$rep.json 2> $OUT/b_${T}_$rep.err || { echo "bench $T failed"; tail -20 $OUT/b_${T}_$rep.err; exit 1; }
    echo "k16_bf16 $T: $(grep ms/step $OUT/b_${T}_$rep.err)"
  done
done
