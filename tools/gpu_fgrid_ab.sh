#!/bin/bash
# Forward workgroup cap (FM_FWD_GRID) sweep, alternating (default: 4096 = fill_grid cap).
set -o pipefail
TAG=${1:-fgrid_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
for rep in 1 2; do
  for PV in "k64 0 1024 2048 3072" "k16_bf16 0 1024 2048" "k128_fp8_ftrl 0 1024 2048"; do
    set -- $PV; P=$1; shift
    for GC in "$@"; do
      FM_FWD_GRID=$GC timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 5 > $OUT/b_${P}_$GC.json 2> $OUT/b_${P}_$GC.err || { echo "bench $P failed"; tail -20 $OUT/b_${P}_$GC.err; exit 1; }
      echo "rep$rep $P fwd_grid=$GC: $(grep ms/step $OUT/b_${P}_$GC.err)"
    done
  done
done
