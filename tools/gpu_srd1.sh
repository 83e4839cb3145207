set -o pipefail
cd $GRAFT_REPO_ROOT
export FM_NO_AUTOBUILD=1
mkdir -p gpurun_out/srd1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_dist_gpu_relay.py > gpurun_out/srd1/pytest.log 2>&1 || { tail -40 gpurun_out/srd1/pytest.log; exit 1; }
tail -3 gpurun_out/srd1/pytest.log
bash tools/gpu_ab.sh srd1 "FM_SELF_ROWS=0|--mode shard --prefetch-rows on --overlap-grads on" "|--mode shard --prefetch-rows on --overlap-grads on" "FM_SELF_ROWS=0|--mode shard" "|--mode shard" "|" "FM_SELF_ROWS=0|--mode shard --prefetch-rows on --overlap-grads on" "|--mode shard --prefetch-rows on --overlap-grads on"
