#!/bin/bash
# Fused loss sum (chunk kernel workgroup 0): tests + A/B; PMC passes of the default step; MFMA counters (hot rows).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r3s2f
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
timeout -k 10 500 python -u -m pytest tests/test_step_gpu.py tests/test_production_schedule_gpu.py tests/test_kernels.py tests/test_fp8_gpu.py tests/test_global_bias.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_ab.sh r3s2f_ab "FM_FUSED_LOSS=0" "FM_FUSED_LOSS=1" "FM_FUSED_LOSS=0" "FM_FUSED_LOSS=1" "FM_FUSED_LOSS=0|--preset k16_bf16" "FM_FUSED_LOSS=1|--preset k16_bf16" || exit 1
bash tools/gpu_pmc.sh r3s2f_pmc || exit 1
FM_HOT_ROWS=1 bash tools/gpu_pmc_mfma.sh r3s2f_mfma || exit 1
