#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-split}
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for V in "off off" "off on" "on on"; do
  set -- $V
  timeout -k 10 300 python bench.py --mode shard --prefetch-rows $1 --overlap-grads $2 --steps 40 --warmup 10 > $OUT/b_$1_$2_$rep.json 2> $OUT/b_$1_$2_$rep.err || { echo "bench failed"; tail -20 $OUT/b_$1_$2_$rep.err; exit 1; }
  echo "prefetch=$1 split=$2: $(grep ms/step $OUT/b_$1_$2_$rep.err)"
done
done
