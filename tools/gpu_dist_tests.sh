#!/bin/bash
# Distributed-path GPU tests (relay ranks on one GPU, RCCL at world 1, production schedules, shard eval).
set -o pipefail
export FM_NO_AUTOBUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/dist_tests
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu_relay.py tests/test_dist_gpu.py tests/test_production_schedule_gpu.py tests/test_shard_eval.py -x -v --timeout 200 --timeout-method thread > $R/gpurun_out/dist_tests/t.log 2>&1
rc=$?
tail -5 $R/gpurun_out/dist_tests/t.log
exit $rc
