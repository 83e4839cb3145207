#!/bin/bash
# fp8 row norms + scaled conversion: fp8 / precision tests, then same-box A/B against ab/head
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4i
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_precision_parity_gpu.py tests/test_step_gpu.py tests/test_production_schedule_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag dir
  (cd $3 && timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err) || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k128_fp8_ftrl k128_ftrl; do
  for rep in 1 2 3; do
    run $P head $R/ab/head || exit 1
    run $P new $R || exit 1
  done
done
# row-sharded step at world 1: chunk workgroups per CU (the local step's cap is off there by default)
for rep in 1 2; do
  for n in 0 3; do
    FM_CHUNK_WG_PER_CU=$n timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --steps 30 --warmup 5 > $OUT/shard_wg$n.json 2> $OUT/shard_wg$n.err || { echo "shard bench failed"; tail -20 $OUT/shard_wg$n.err; exit 1; }
    echo "shard wg$n: $(grep ms/step $OUT/shard_wg$n.err)"
  done
done
