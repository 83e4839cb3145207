#!/bin/bash
# fp8 chunk kernel without the piece support: GPU tests touching fp8 tables, then a same-box A/B.
set -o pipefail
export FM_NO_AUTOBUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/flat
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_production_schedule_gpu.py tests/test_precision_parity_gpu.py tests/test_step_gpu.py tests/test_dist_gpu_relay.py -x -v --timeout 200 --timeout-method thread > $R/gpurun_out/flat/t.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/flat/t.log; exit 1; }
tail -1 $R/gpurun_out/flat/t.log
bash tools/gpu_ab.sh flat_ab "FM_CHUNK_FLAT=0|--preset k128_fp8_ftrl" "FM_CHUNK_FLAT=1|--preset k128_fp8_ftrl" "FM_CHUNK_FLAT=0|--preset k128_fp8_ftrl" "FM_CHUNK_FLAT=1|--preset k128_fp8_ftrl" "|--preset k128_ftrl" "|--preset k128_ftrl" "|" || exit 1
