#!/bin/bash
# Full GPU pass: test suite, smoke, every bench preset, sharded step at world 1 (RCCL),
# kernel profile of the headline bench.  usage: tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for P in k64 k64_bf16 k16_bf16 k128_ftrl k128_fp8_ftrl k64_dp_dense; do
  timeout -k 10 300 python bench.py --preset $P > $OUT/bench_$P.json 2> $OUT/bench_$P.err || { echo "bench $P failed"; tail -20 $OUT/bench_$P.err; exit 1; }
  echo "$P: $(grep ms/step $OUT/bench_$P.err)"
done
for V in "shard" "shard_bf16wire --comm-dtype bf16"; do
  set -- $V; N=$1; shift
  timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard "$@" > $OUT/bench_$N.json 2> $OUT/bench_$N.err || { echo "bench $N failed"; tail -20 $OUT/bench_$N.err; exit 1; }
  echo "$N: $(grep ms/step $OUT/bench_$N.err)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/kernel_summary.txt
python3 $R/tools/timeline.py $OUT/prof/run_kernel_trace.csv fm_fwd_kernel > $OUT/timeline.txt
head -12 $OUT/kernel_summary.txt
