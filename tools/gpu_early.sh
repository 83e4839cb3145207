#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-early}
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for PF in off on; do
  FM_PREFETCH=$PF timeout -k 10 300 python bench.py --mode shard --prefetch-rows $PF --steps 40 --warmup 10 > $OUT/b_${PF}_$rep.json 2> $OUT/b_${PF}_$rep.err || { echo "bench failed"; tail -20 $OUT/b_${PF}_$rep.err; exit 1; }
  echo "prefetch=$PF: $(grep ms/step $OUT/b_${PF}_$rep.err)"
done
done
