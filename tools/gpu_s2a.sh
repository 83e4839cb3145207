#!/bin/bash
# Session check: bucket-sort dedup tests, GPU suite + bench, dedup A/B, kernel profiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r3s2
export FM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_dedup_sort_gpu.py -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r3s2/dedup_sort.log 2>&1 || { echo "dedup sort tests failed"; tail -40 $R/gpurun_out/r3s2/dedup_sort.log; exit 1; }
tail -3 $R/gpurun_out/r3s2/dedup_sort.log
bash tools/gpu_ab.sh r3s2_ab "FM_DEDUP_SORT=onesweep" "FM_DEDUP_SORT=bucket" "FM_DEDUP_SORT=onesweep FM_HOT_ROWS=0" "FM_DEDUP_SORT=bucket FM_HOT_ROWS=0" "FM_DEDUP_SORT=onesweep" "FM_DEDUP_SORT=bucket" || exit 1
bash tools/gpu_final_prof.sh r3s2_prof || exit 1
FM_DEDUP_SORT=onesweep bash tools/gpu_final_prof.sh r3s2_prof_os || exit 1
bash tools/gpu_round.sh r3s2 || exit 1
