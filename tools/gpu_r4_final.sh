#!/bin/bash
# round-4 end check: GPU suite + smoke + default bench + sharded bench (tools/gpu_round.sh), every
# preset, and the sharded step at world 1 for the k16 / k128 fp8 presets
set -o pipefail
TAG=${1:-r4_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
bash tools/gpu_round.sh $TAG || exit 1
cd $R
export FM_NO_AUTOBUILD=1
for P in k64_bf16 k16_bf16 k128_ftrl k128_fp8_ftrl k64_dp_dense; do
  timeout -k 10 300 python bench.py --preset $P --steps 30 --warmup 5 > $OUT/bench_$P.json 2> $OUT/bench_$P.err || { echo "bench $P failed"; tail -20 $OUT/bench_$P.err; exit 1; }
  echo "$P: $(grep ms/step $OUT/bench_$P.err)"
done
for P in k16_bf16 k128_fp8_ftrl; do
  timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --preset $P --mode shard --steps 30 --warmup 5 > $OUT/bench_shard_$P.json 2> $OUT/bench_shard_$P.err || { echo "shard bench $P failed"; tail -20 $OUT/bench_shard_$P.err; exit 1; }
  echo "shard $P: $(grep ms/step $OUT/bench_shard_$P.err)"
done
# the local forward's k64 occupancy choice against the previous one (FM_HIP_VARIANT=fu10w4), if built
if [ -f fast_tffm_amd/_native/_fm_hip_fu10w4.cpython-310-x86_64-linux-gnu.so ]; then
  for rep in 1 2; do
    for V in "" fu10w4; do
      for P in k64 k64_bf16; do
        FM_HIP_VARIANT=$V timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/ab_${P}_${V:-new}.json 2> $OUT/ab_${P}_${V:-new}.err || { echo "ab $P $V failed"; exit 1; }
        echo "$P ${V:-new}: $(grep ms/step $OUT/ab_${P}_${V:-new}.err)"
      done
    done
  done
fi
