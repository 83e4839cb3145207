#!/bin/bash
# First GPU bring-up: kernel numerics, smoke, single-GPU bench at a few batch sizes.
set -o pipefail
mkdir -p gpurun_out
export FM_NO_AUTOBUILD=1
rocm-smi --showmeminfo vram > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
for B in 65536 131072 262144; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch $B > gpurun_out/bench_B$B.json 2> gpurun_out/bench_B$B.err || { echo "bench B=$B failed"; tail -20 gpurun_out/bench_B$B.err; exit 1; }
  tail -2 gpurun_out/bench_B$B.err
done
