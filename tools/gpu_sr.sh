#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-sr}
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for P in k64 k16_bf16 k128_fp8_ftrl; do
  timeout -k 10 300 python bench.py --preset $P > $OUT/bench_$P.json 2> $OUT/bench_$P.err || { echo "bench $P failed"; tail -20 $OUT/bench_$P.err; exit 1; }
  echo "$P: $(grep ms/step $OUT/bench_$P.err)"
done
