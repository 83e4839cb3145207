#!/bin/bash
# hot-row workgroup combine beside the lane-group combine (FM_BWD_BIG_FORK): step tests, then A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4p
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py tests/test_fp8_gpu.py tests/test_production_schedule_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag env...
  local P=$1 T=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { echo "bench $P $T failed"; tail -20 $OUT/b_${P}_$T.err; return 1; }
  echo "$P $T: $(grep ms/step $OUT/b_${P}_$T.err)"
}
for P in k64 k16_bf16 k128_fp8_ftrl k64_bf16; do
  for rep in 1 2; do
    run $P fork FM_BWD_BIG_FORK=1 || exit 1
    run $P serial FM_BWD_BIG_FORK=0 || exit 1
  done
done
