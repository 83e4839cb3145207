#!/bin/bash
# stored row norms for every dtype (+ fp8 power-of-two scales / scaled conversion): full GPU suite,
# then same-box A/B against ab/head (the commit before the norms)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4j
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # preset tag dir
  (cd $3 && timeout -k 10 200 python bench.py --preset $1 --steps 40 --warmup 8 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err) || { echo "bench $1 $2 failed"; tail -20 $OUT/b_$1_$2.err; return 1; }
  echo "$1 $2: $(grep ms/step $OUT/b_$1_$2.err)"
}
for P in k64 k128_fp8_ftrl k128_ftrl k64_bf16 k16_bf16; do
  for rep in 1 2; do
    run $P head $R/ab/head || exit 1
    run $P new $R || exit 1
  done
done
# row-sharded step at world 1: wire norms (new) vs none (fwdnonorm) vs ab/head; chunk workgroups per CU
shard() {  # tag dir variant env...
  local T=$1 D=$2 V=$3; shift 3
  (cd $D && env FM_HIP_VARIANT=$V "$@" timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --steps 30 --warmup 5 > $OUT/shard_$T.json 2> $OUT/shard_$T.err) || { echo "shard bench $T failed"; tail -20 $OUT/shard_$T.err; return 1; }
  echo "shard $T: $(grep ms/step $OUT/shard_$T.err)"
}
for rep in 1 2; do
  shard head $R/ab/head "" X=1 || exit 1
  shard new $R "" X=1 || exit 1
  shard nonorm $R fwdnonorm X=1 || exit 1
  shard wg3 $R "" FM_CHUNK_WG_PER_CU=3 || exit 1
done
