#!/bin/bash
# same-box A/B: the committed tree (ab/head, a git worktree of HEAD with its own build) against the
# working tree, its bwdgen variant (general chunk kernel) and fwdgen variant (general forward)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4d
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_fp8_gpu.py tests/test_parse_gpu.py tests/test_production_schedule_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag dir variant
  (cd $3 && FM_HIP_VARIANT=$4 timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err) || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; exit 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k64 k128_fp8_ftrl k64_bf16 k16_bf16; do
  for rep in 1 2; do
    run $P head $R/ab/head "" || exit 1
    run $P new $R "" || exit 1
    run $P bwdgen $R bwdgen || exit 1
    run $P fwdgen $R fwdgen || exit 1
    [ $P = k128_fp8_ftrl ] && { run $P fwdfold $R fwdfold || exit 1; }
  done
done
