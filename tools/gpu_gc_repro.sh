#!/bin/bash
# Reproduce the GC-time abort after the lookahead graph-ring test (stderr unbuffered, -s).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gcab
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
timeout -k 10 200 python -X faulthandler -u -m pytest -s -x -v --timeout 120 --timeout-method thread tests/test_step_gpu.py -k "graph_ring or stochastic or local_lookahead" > $OUT/a.log 2>&1; echo "rc=$?"
grep -v "^  File" $OUT/a.log | tail -40
