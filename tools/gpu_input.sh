#!/bin/bash
# Input paths on the GPU box: loader throughput (CPU parse / GPU tokenizer / .fmb cache)
# and end-to-end run.py train on the reference's sample workload shape.
# usage: tools/gpu_input.sh <tag>
set -o pipefail
TAG=${1:-input}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 400 python -u tools/bench_input.py --skip-python --threads 16 --dir /tmp/fm_in > $OUT/bench_input.txt 2>&1 || { echo "bench_input failed"; tail -30 $OUT/bench_input.txt; exit 1; }
cat $OUT/bench_input.txt
timeout -k 10 500 python -u tools/bench_train_e2e.py --threads 16 --epochs 6 --dir /tmp/fm_e2e > $OUT/bench_e2e.txt 2>&1 || { echo "bench_e2e failed"; tail -30 $OUT/bench_e2e.txt; exit 1; }
cat $OUT/bench_e2e.txt
