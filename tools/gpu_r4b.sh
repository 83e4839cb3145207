#!/bin/bash
# forward specialization: GPU suite, then same-box A/B (specialized local forward vs the general one)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for P in k64 k128_fp8_ftrl k16_bf16; do
  for V in "" fwdgen "" fwdgen; do
    FM_HIP_VARIANT=$V timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/b_${P}_$V.json 2> $OUT/b_${P}_$V.err || { echo "bench $P $V failed"; tail -20 $OUT/b_${P}_$V.err; exit 1; }
    echo "$P variant=${V:-specialized}: $(grep ms/step $OUT/b_${P}_$V.err)"
  done
done
