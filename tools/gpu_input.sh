#!/bin/bash
# Input-path checks and throughput: GPU tokenizer tests, reader stage timing, file-fed e2e training.
set -o pipefail
TAG=${1:-input}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FM_NO_AUTOBUILD=1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parse_gpu.py tests/test_loader_slots.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_loader.py --threads 16 --epochs 5 > $OUT/loader.txt 2>&1 || { tail -20 $OUT/loader.txt; exit 1; }
cat $OUT/loader.txt
timeout -k 10 300 python -u tools/bench_gpu_parse_stages.py --threads 16 > $OUT/stages.txt 2>&1 || { tail -20 $OUT/stages.txt; exit 1; }
cat $OUT/stages.txt
# (8 parse threads: one per physical core of the box's 16-CPU share -- the sweep in profiles/r5/e2e.txt)
timeout -k 10 600 python -u tools/bench_train_e2e.py --lines 250000 --files 4 --epochs 8 --threads 8 > $OUT/e2e.txt 2>&1 || { tail -20 $OUT/e2e.txt; exit 1; }
cat $OUT/e2e.txt
