#!/bin/bash
# chunk workgroups per CU (FM_CHUNK_WG_PER_CU, capped through dynamic LDS) sweep per preset
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4h
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd $R
run() {  # preset tag env...
  local P=$1 T=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --preset $P --steps 40 --warmup 8 > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { echo "bench $P $T failed"; tail -20 $OUT/b_${P}_$T.err; return 1; }
  echo "$P $T: $(grep ms/step $OUT/b_${P}_$T.err)"
}
sweep() {  # preset values...
  local P=$1; shift
  for rep in 1 2; do for n in "$@"; do run $P wg$n FM_CHUNK_WG_PER_CU=$n || return 1; done; done
}
sweep k64 0 2 3 4 && sweep k64_bf16 0 3 4 && sweep k16_bf16 0 2 3 4 && sweep k128_fp8_ftrl 0 4 6 && sweep k128_ftrl 0 4
