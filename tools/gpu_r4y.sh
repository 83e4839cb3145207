#!/bin/bash
# sharded fp8 forward with stored row norms (wire tail word 2): fp8 / sharded GPU tests, then the EMIT
# path (FM_SHARD_W1_LOCAL=0, the per-rank compute of N>1) vs the fwdshnonorm variant, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4y
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_dist_gpu_relay.py tests/test_dist_gpu.py tests/test_shard_eval.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 FM_SHARD_W1_LOCAL=0
i=0
for rep in 1 2; do
  for V in base fwdshnonorm; do
    T=$V; [ $V = base ] && V=""
    i=$((i+1)); export MASTER_PORT=$((29660+i))
    FM_HIP_VARIANT=$V timeout -k 10 300 python bench.py --gpus 1 --mode shard --preset k128_fp8_ftrl --steps 40 --warmup 8 > $OUT/v$i.json 2> $OUT/v$i.err || { echo "shard bench failed"; tail -20 $OUT/v$i.err; exit 1; }
    echo "[EMIT k128 fp8 $T] $(grep ms/step $OUT/v$i.err)"
  done
done
