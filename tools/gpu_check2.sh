#!/bin/bash
# Profile the single-GPU step and exercise the RCCL (world=1) exchange paths.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof1.log 2>&1 || { echo "rocprof failed"; tail -30 $R/gpurun_out/prof1.log; exit 1; }
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode shard > gpurun_out/bench_shard_w1.json 2> gpurun_out/bench_shard_w1.err || { echo "shard w1 failed"; tail -30 gpurun_out/bench_shard_w1.err; exit 1; }
tail -1 gpurun_out/bench_shard_w1.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --preset k64_dp_dense > gpurun_out/bench_dpdense_w1.json 2> gpurun_out/bench_dpdense_w1.err || { echo "dp_dense failed"; tail -30 gpurun_out/bench_dpdense_w1.err; exit 1; }
tail -1 gpurun_out/bench_dpdense_w1.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --preset k16_bf16 > gpurun_out/bench_k16bf16.json 2> gpurun_out/bench_k16bf16.err || { echo "k16 failed"; tail -30 gpurun_out/bench_k16bf16.err; exit 1; }
tail -1 gpurun_out/bench_k16bf16.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --preset k128_ftrl > gpurun_out/bench_k128ftrl.json 2> gpurun_out/bench_k128ftrl.err || { echo "k128 failed"; tail -30 gpurun_out/bench_k128ftrl.err; exit 1; }
tail -1 gpurun_out/bench_k128ftrl.err
find $R/gpurun_out/prof1 -name "*stats*" | head
