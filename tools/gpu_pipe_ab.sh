#!/bin/bash
# Software-pipelined chunk kernel (FM_CHUNK_PIPE): GPU tests, then an alternating same-box A/B
# of the 16-lane presets (local and sharded) and a kernel profile.
# usage: tools/gpu_pipe_ab.sh <tag>
set -o pipefail
TAG=${1:-pipe_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_dist_gpu.py tests/test_dist_gpu_relay.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest_pipe.log | head -30; tail -30 $OUT/pytest_pipe.log; exit 1; }
tail -1 $OUT/pytest_pipe.log
for rep in 1 2 3; do
  for P in k64 k64_bf16 k64_dp_dense; do
    for F in 0 1; do
      FM_CHUNK_PIPE=$F timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$F.json 2> $OUT/b_${P}_$F.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$F.err; exit 1; }
      echo "rep$rep $P chunk_pipe=$F: $(grep ms/step $OUT/b_${P}_$F.err)"
    done
  done
  for F in 0 1; do
    FM_CHUNK_PIPE=$F timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode shard --prefetch-rows on --steps 40 --warmup 5 > $OUT/b_shard_$F.json 2> $OUT/b_shard_$F.err || { echo "shard bench failed"; tail -20 $OUT/b_shard_$F.err; exit 1; }
    echo "rep$rep shard(early rows on) chunk_pipe=$F: $(grep ms/step $OUT/b_shard_$F.err)"
  done
done
cd /tmp && export TMPDIR=/tmp
for F in 0 1; do
  FM_CHUNK_PIPE=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$F -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $OUT/prof$F.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof$F.log; exit 1; }
  python3 $R/tools/kstats.py $OUT/prof$F/run_kernel_stats.csv 25 > $OUT/kernel_summary_pipe$F.txt
  grep -h "chunk\|fm_fwd" $OUT/kernel_summary_pipe$F.txt
  rm -f $OUT/prof$F/run_kernel_trace.csv
done
