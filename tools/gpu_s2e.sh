#!/bin/bash
# Split chunk walk: tests, A/B, timeline; gather roofline microbenchmark; PMC passes of the default step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r3s2e
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
FM_BWD_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests2.log 2>&1 || { echo "tests (split 2) failed"; tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
timeout -k 10 500 python -u -m pytest tests/test_step_gpu.py tests/test_production_schedule_gpu.py tests/test_hot_rows_gpu.py tests/test_dedup_sort_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_ab.sh r3s2e_ab "FM_BWD_SPLIT=0" "FM_BWD_SPLIT=1" "FM_BWD_SPLIT=2" "FM_BWD_SPLIT=0" "FM_BWD_SPLIT=1" "FM_BWD_SPLIT=2" "FM_BWD_SPLIT=0|--preset k16_bf16" "FM_BWD_SPLIT=1|--preset k16_bf16" "FM_BWD_SPLIT=0|--preset k128_fp8_ftrl" "FM_BWD_SPLIT=1|--preset k128_fp8_ftrl" || exit 1
timeout -k 10 120 tools/bench_gather > $OUT/gather.txt 2>&1 || { echo "bench_gather failed"; cat $OUT/gather.txt; exit 1; }
cat $OUT/gather.txt
bash tools/gpu_final_prof.sh r3s2e_prof || exit 1
for i in 1 2 3 4 5; do echo "pmc pass $i" >> $OUT/progress.txt; done
bash tools/gpu_pmc.sh r3s2e_pmc || exit 1
