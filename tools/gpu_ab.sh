#!/bin/bash
# A/B of step variants on one box (1 GPU, default bench config unless args given).
# usage: tools/gpu_ab.sh <tag> "ENV=.. ENV=..|bench args" "ENV=..|bench args" ...
# (the part before '|' is the environment, after it extra bench.py arguments)
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
  ENVS=${V%%|*}
  ARGS=""
  [[ "$V" == *"|"* ]] && ARGS=${V#*|}
  env FM_AB_RUN=$i $ENVS timeout -k 10 200 python bench.py --steps 40 --warmup 5 $ARGS > $OUT/v$i.json 2> $OUT/v$i.err || { echo "variant $V failed"; tail -20 $OUT/v$i.err; exit 1; }
  echo "[$V] $(grep ms/step $OUT/v$i.err)"
done
