#!/bin/bash
# final-code GPU suite, then the chunk-grid x workgroups-per-CU sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4k
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag env...
  local P=$1 T=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { echo "bench $P $T failed"; tail -20 $OUT/b_${P}_$T.err; return 1; }
  echo "$P $T: $(grep ms/step $OUT/b_${P}_$T.err)"
}
for rep in 1 2; do
  for g in 2304 3072 3840 5120; do run k64 g$g FM_CHUNK_GRID=$g || exit 1; done
  for g in 384 512 768 1024; do run k16_bf16 g$g FM_CHUNK_GRID=$g || exit 1; done
  for g in 2048 4096; do run k128_fp8_ftrl g${g}w4 FM_CHUNK_GRID=$g FM_CHUNK_WG_PER_CU=4 || exit 1; done
  run k128_fp8_ftrl g4096w0 FM_CHUNK_GRID=4096 || exit 1
  run k128_fp8_ftrl base X=1 || exit 1
done
