#!/bin/bash
# MFMA / VALU / LDS counters (kernel trace only), summarised by tools/pmc_summary.py
# (MFMA% = sum SQ_VALU_MFMA_BUSY_CYCLES / (per-instance GRBM_GUI_ACTIVE x 1024 SIMDs), as rocprof's MfmaUtil).
# usage: tools/gpu_pmc_mfma.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc_mfma}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
# counter passes serialise every dispatch (the synthetic pool's ~20k small generation kernels
# included: --pool 3 keeps that short); a heartbeat file under gpurun_out/ marks progress
( while sleep 30; do date >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
i=0
for CTRS in "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph 0 --pool 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT | tee $OUT/pmc_summary.txt
# per-dispatch CSVs can pass gpurun's 64 MiB merge-back limit: keep the summary only
find $OUT -name '*.csv' -delete
