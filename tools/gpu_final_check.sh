#!/bin/bash
# Round-end check on one box: GPU suite + smoke + default bench + sharded bench, every preset, PMC passes.
set -o pipefail
bash tools/gpu_round.sh r3_final || exit 1
bash tools/gpu_presets.sh r3_final_presets || exit 1
bash tools/gpu_pmc.sh r3_final_pmc || exit 1
