#!/bin/bash
# Same-box A/B of the chunk kernel with / without the fused loss sum compiled in (build variant nofl).
set -o pipefail
bash tools/gpu_ab.sh r3_fl_ab "FM_HIP_VARIANT=nofl FM_FUSED_LOSS=0" "FM_FUSED_LOSS=1" "FM_FUSED_LOSS=0" "FM_HIP_VARIANT=nofl FM_FUSED_LOSS=0" "FM_FUSED_LOSS=1" "FM_HIP_VARIANT=nofl FM_FUSED_LOSS=0|--preset k64_dp_dense" "FM_FUSED_LOSS=1|--preset k64_dp_dense" "FM_HIP_VARIANT=nofl FM_FUSED_LOSS=0|--preset k128_ftrl" "FM_FUSED_LOSS=1|--preset k128_ftrl" || exit 1
