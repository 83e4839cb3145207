#!/bin/bash
# Full GPU test suite, then a bench A/B (tools/gpu_ab.sh variants).
# usage: tools/gpu_suite_ab.sh <tag> "ENV|args" ...
set -o pipefail
TAG=${1:-suite}; shift
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export FM_NO_AUTOBUILD=1
mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
[ $# -gt 0 ] && bash tools/gpu_ab.sh $TAG "$@"
exit 0
