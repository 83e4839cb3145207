#!/bin/bash
# Stochastic-rounding cost A/B per preset.  usage: tools/gpu_sr_ab.sh <tag> <preset>...
set -o pipefail
TAG=${1:-srab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for p in "$@"; do
    for sr in on off; do
      timeout -k 10 200 python bench.py --preset $p --steps 50 --warmup 10 --stochastic-rounding $sr > /dev/null 2> $OUT/err.txt || { echo "bench failed"; tail -20 $OUT/err.txt; exit 1; }
      echo "sr=$sr preset=$p rep=$rep: $(grep ms/step $OUT/err.txt)" | tee -a $OUT/ab.txt
    done
  done
done
