#!/bin/bash
# Memory-system diagnosis of the default step (1 GPU):
#  1. table-size sweep (same batch shape, fewer hashed slots -> fewer pages / less HBM spread)
#  2. PMC passes (kernel trace only, one block budget per pass): TLB, TA/TCP stalls and
#     L2->TCP latency, SQ instruction mix, L2 hits and fabric bytes.
# usage: tools/gpu_diag.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-diag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for S in ${SIZES-125000000 31250000 8000000 2000000}; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --slots-per-gpu $S "$@" > $OUT/size_$S.json 2> $OUT/size_$S.err || { echo "size $S failed"; tail -20 $OUT/size_$S.err; exit 1; }
  echo "slots $S: $(grep ms/step $OUT/size_$S.err)"
done
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT GRBM_GUI_ACTIVE" \
            "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM SQ_WAVE_CYCLES" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE" \
            "WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum" \
            "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "fm::|rocprim" --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; break; }
  python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
