#!/bin/bash
# sharded step at world 1: LOCAL-mode backward (default) vs the EMIT path (FM_SHARD_W1_LOCAL=0),
# alternating on one box, k64 fp32 / k16 bf16 / k128 fp8; shard GPU tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4v
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_owner_counts_gpu.py tests/test_dist_gpu.py tests/test_production_schedule_gpu.py tests/test_dist_gpu_relay.py tests/test_teardown_gpu.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
i=0
for P in "" "--preset k16_bf16" "--preset k128_fp8_ftrl"; do
  for rep in 1 2; do
    for V in 1 0; do
      i=$((i+1)); export MASTER_PORT=$((29570+i))
      FM_SHARD_W1_LOCAL=$V timeout -k 10 300 python bench.py --gpus 1 --mode shard $P --steps 40 --warmup 8 > $OUT/v$i.json 2> $OUT/v$i.err || { echo "shard bench failed"; tail -20 $OUT/v$i.err; exit 1; }
      echo "[shard $P local_w1=$V] $(grep ms/step $OUT/v$i.err)"
    done
  done
done
