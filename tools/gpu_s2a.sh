#!/bin/bash
set -o pipefail
bash tools/gpu_round.sh r3s2 || exit 1
bash tools/gpu_ab.sh r3s2_hot "FM_HOT_ROWS=0" "FM_HOT_ROWS=1" "FM_HOT_ROWS=0" "FM_HOT_ROWS=1" || exit 1
bash tools/gpu_final_prof.sh r3s2_prof || exit 1
FM_HOT_ROWS=0 bash tools/gpu_final_prof.sh r3s2_prof_nohot || exit 1
