#!/bin/bash
# PMC counter passes over a short bench run (kernel-trace only: no sys/runtime trace with --pmc).
# usage: tools/gpu_pmc.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift
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
for CTRS in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph 0 --pool 3 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT | tee $OUT/pmc_summary.txt
# per-dispatch CSVs can pass gpurun's 64 MiB merge-back limit: keep the summary only
find $OUT -name '*.csv' -delete
