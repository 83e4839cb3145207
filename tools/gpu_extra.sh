#!/bin/bash
# Diagnostics on one box after the round check: side-chain cost split, PMC counter passes of the
# default step (memory roofline inputs), MFMA counters with the dense-row MFMA backward on.
# usage: tools/gpu_extra.sh <tag>
set -o pipefail
TAG=${1:-extra}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python tools/side_chain_cost.py > $OUT/side_chain.txt 2>&1 || { echo "side chain failed"; tail -20 $OUT/side_chain.txt; exit 1; }
grep side_chain $OUT/side_chain.txt
bash tools/gpu_pmc.sh ${TAG}_pmc || exit 1
FM_DENSE_BWD=1 bash tools/gpu_pmc_mfma.sh ${TAG}_mfma || exit 1
