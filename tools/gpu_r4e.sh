#!/bin/bash
# per-kernel time: committed tree (ab/head) vs working tree, k128 fp8 FTRL, k16 bf16 and k64 fp32
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4e
mkdir -p $OUT
export FM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for P in k16_bf16; do
  for T in head new bwdgen fwdgen; do
    D=$R; [ $T = head ] && D=$R/ab/head
    V=""; [ $T = bwdgen ] && V=bwdgen; [ $T = fwdgen ] && V=fwdgen
    cd $D && FM_HIP_VARIANT=$V timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${P}_$T -o run -- python3 bench.py --preset $P --steps 30 --warmup 5 > $OUT/b_${P}_$T.json 2> $OUT/b_${P}_$T.err || { echo "prof $P $T failed"; tail -20 $OUT/b_${P}_$T.err; exit 1; }
    echo "$P $T: $(grep ms/step $OUT/b_${P}_$T.err)"
    find $OUT/prof_${P}_$T -type f -printf "%s %p\n" > $OUT/files_${P}_$T.txt
    python3 $R/tools/kstats.py $OUT/prof_${P}_$T 35 > $OUT/kstats_${P}_$T.txt || true
    find $OUT/prof_${P}_$T -type f -name "*kernel_trace.csv" -delete
  done
done
