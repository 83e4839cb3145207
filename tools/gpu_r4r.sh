#!/bin/bash
# chunk backward r1 rows in flight for 32-lane rows (default 12 vs 8 / 10 / 14) on k128 fp8 / bf16
# FTRL, and the k64 local forward with 2 row groups in flight at 7 waves/SIMD (fu2w7)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4r
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag variant
  FM_HIP_VARIANT=$3 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k128_fp8_ftrl k128_ftrl; do
  for rep in 1 2; do
    for V in base cu32_8 cu32_10 cu32_14; do
      T=$V; [ $V = base ] && V=""
      run $P $T "$V" || exit 1
    done
  done
done
for rep in 1 2 3; do
  run k64 base "" || exit 1
  run k64 fu2w7 fu2w7 || exit 1
done
