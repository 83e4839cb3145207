#!/bin/bash
# chunk-backward specialization: backward/step GPU tests, then same-box A/B of the specialized
# build against FM_HIP_VARIANT=bwdgen (general chunk kernel) and fwdgen (general forward)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4c
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_fp8_gpu.py tests/test_production_schedule_gpu.py tests/test_precision_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for P in k64 k128_fp8_ftrl k16_bf16 k64_bf16; do
  for V in "" bwdgen fwdgen "" bwdgen fwdgen; do
    FM_HIP_VARIANT=$V timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/b_${P}_$V.json 2> $OUT/b_${P}_$V.err || { echo "bench $P $V failed"; tail -20 $OUT/b_${P}_$V.err; exit 1; }
    echo "$P variant=${V:-specialized}: $(grep ms/step $OUT/b_${P}_$V.err)"
  done
done
