#!/bin/bash
# round-4 session check: hd dedup (tests, chain alone, step A/B, kernel profile), then the complete
# PMC tables of the k64 fp32 and k128 fp8 FTRL steps
set -o pipefail
bash tools/gpu_hd.sh hd3 || exit 1
bash tools/gpu_pmc_full.sh pmc_k64 || exit 1
bash tools/gpu_pmc_full.sh pmc_k128fp8 --preset k128_fp8_ftrl || exit 1
