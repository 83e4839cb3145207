#!/usr/bin/env python3
"""Per-kernel MFMA / LDS / L2 counter table from tools/gpu_pmc_mfma.sh passes (averaged per dispatch)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        if "fm::" not in name:
            continue
        acc[name.split("(")[0][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        if "fm::" not in name:
            continue
        dur[name.split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def avg(c, n):
    v = c.get(n)
    return sum(v) / len(v) if v else float("nan")


print(f"{'kernel':60s} {'us':>7s} {'MFMA_F32':>10s} {'MFMAbusy%':>9s} {'LDSconf%':>8s} {'L2hit%':>7s} {'FETCH_MB':>9s}")
for k, c in sorted(acc.items(), key=lambda kv: -sum(dur.get(kv[0], [0]))):
    d = sorted(dur.get(k, [0]))
    us = d[len(d) // 2] if d else 0
    busy = avg(c, "SQ_VALU_MFMA_BUSY_CYCLES") / max(avg(c, "SQ_BUSY_CYCLES"), 1) * 100
    lds = avg(c, "SQ_LDS_BANK_CONFLICT") / max(avg(c, "SQ_LDS_IDX_ACTIVE"), 1) * 100
    hit, miss = avg(c, "TCC_HIT_sum"), avg(c, "TCC_MISS_sum")
    print(f"{k:60s} {us:7.1f} {avg(c, 'SQ_INSTS_VALU_MFMA_F32'):10.0f} {busy:9.1f} {lds:8.1f} "
          f"{100 * hit / max(hit + miss, 1):7.1f} {avg(c, 'FETCH_SIZE') / 1024:9.1f}")
