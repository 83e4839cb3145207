#!/bin/bash
# Same-box A/B of this tree against ab_old/ -- a copy of an earlier commit with its own in-tree build:
#   rm -rf ab_old && mkdir ab_old && git archive <commit> | tar -x -C ab_old
#   (cd ab_old && python -c "import __graft_entry__ as g; g.build()")
# then: gpurun -- 'bash tools/gpu_ab_tree.sh'.  GPU tests on this tree first, then the default / k16 bf16 /
# k128 fp8 FTRL / default presets and the world-1 EMIT step, alternating new / old.  (Delete ab_old/ after:
# every gpurun call uploads it.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cmb
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for args in "" "--preset k16_bf16" "--preset k128_fp8_ftrl" ""; do
  for side in new old; do
    i=$((i+1))
    if [ $side = new ]; then D=$R; else D=$R/ab_old; fi
    (cd $D && timeout -k 10 200 python bench.py --steps 40 --warmup 5 $args > $OUT/r$i.json 2> $OUT/r$i.err) || { echo "run $i failed"; tail -20 $OUT/r$i.err; exit 1; }
    echo "[$side $args] $(grep ms/step $OUT/r$i.err)"
  done
done
for side in new old; do
  i=$((i+1))
  if [ $side = new ]; then D=$R; else D=$R/ab_old; fi
  (cd $D && FM_SHARD_W1_LOCAL=0 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --mode shard > $OUT/r$i.json 2> $OUT/r$i.err) || { echo "run $i failed"; tail -20 $OUT/r$i.err; exit 1; }
  echo "[$side EMIT] $(grep ms/step $OUT/r$i.err)"
done
