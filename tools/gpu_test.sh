#!/bin/bash
# GPU test suite only (optionally a subset): tools/gpu_test.sh <tag> [pytest args...]
set -o pipefail
TAG=${1:-gpt}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 500 python -m pytest tests -m gpu -q "$@" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -40 $OUT/pytest_gpu.log
exit $rc
