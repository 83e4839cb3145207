#!/bin/bash
# final-code PMC tables: k64 fp32 and k128 fp8 FTRL steps
set -o pipefail
bash tools/gpu_pmc_full.sh pmc_k64_final || exit 1
bash tools/gpu_pmc_full.sh pmc_k128fp8_final --preset k128_fp8_ftrl || exit 1
