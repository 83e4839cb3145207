#!/bin/bash
# Session batch: loss-stream tests + A/B, isolated dedup chain, PMC roofline passes, MFMA counters (hot rows).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r3s2d
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_production_schedule_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_ab.sh r3s2d_ab "FM_LOSS_STREAM=0" "FM_LOSS_STREAM=1" "FM_LOSS_STREAM=0" "FM_LOSS_STREAM=1" || exit 1
bash tools/gpu_s2c.sh || exit 1
timeout -k 10 200 python tools/gather_roofline.py > $OUT/gather.log 2>&1 || { echo "gather roofline failed"; tail -20 $OUT/gather.log; exit 1; }
grep gather_roofline $OUT/gather.log
bash tools/gpu_pmc.sh r3s2d_pmc > /dev/null || exit 1
cut -c1-200 $R/gpurun_out/r3s2d_pmc/pmc_summary.txt | head -14
FM_HOT_ROWS=1 bash tools/gpu_pmc_mfma.sh r3s2d_mfma > /dev/null || exit 1
cut -c1-200 $R/gpurun_out/r3s2d_mfma/pmc_summary.txt | head -14
