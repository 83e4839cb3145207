#!/bin/bash
# MFMA / LDS counters of the dense-row MFMA backward (FM_DENSE_BWD=1), kernel trace only.
# usage: tools/gpu_pmc_mfma.sh <tag>
set -o pipefail
TAG=${1:-pmc_mfma}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1 FM_DENSE_BWD=1
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_mfma_summary.py $OUT | tee $OUT/pmc_mfma_summary.txt
