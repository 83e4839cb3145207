#!/bin/bash
# Complete PMC table of a bench step (kernel-trace only, one counter pass per run, within the
# per-block limits: <= 8 SQ, <= 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), <= 4 TCP, <= 2 TA, <= 2 GRBM).
# usage: tools/gpu_pmc_full.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmcfull}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
i=0
for CTRS in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" \
            "WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum" \
            "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE TA_TA_BUSY TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_TRANSLATION_MISS TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph 0 --pool 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT | tee $OUT/pmc_summary.txt
find $OUT -name '*.csv' -delete
