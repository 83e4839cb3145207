#!/bin/bash
# A/B of step variants selected by environment variables (1 GPU, default bench config).
# usage: tools/gpu_ab.sh <tag> "ENV=.. ENV=.." "ENV=.." ...
set -o pipefail
TAG=${1:-ab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 200 python bench.py --steps 40 --warmup 5 > $OUT/v$i.json 2> $OUT/v$i.err || { echo "variant $V failed"; tail -20 $OUT/v$i.err; exit 1; }
  echo "[$V] $(grep ms/step $OUT/v$i.err)"
done
