#!/usr/bin/env python3
"""Merge rocprofv3 --pmc counter CSVs (one dir per pass) into a per-kernel table (averaged per dispatch)."""
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
        name = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
        if not name.startswith(("void fm::", "fm::", "void rocprim")):
            continue
        key = name.split("(")[0][:70]
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        if not name.startswith(("void fm::", "fm::", "void rocprim")):
            continue
        key = name.split("(")[0][:70]
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':70s} {'us':>7s} {'L2hit%':>7s} {'FETCH_MB':>9s} {'WRITE_MB':>9s} {'GB/s(f+w)':>9s} {'waitany%':>8s}")
for k, c in sorted(acc.items(), key=lambda kv: -sum(dur.get(kv[0], [0]))):
    d = sorted(dur.get(k, [0]))
    us = d[len(d) // 2] if d else 0
    def avg(n):
        v = c.get(n)
        return sum(v) / len(v) if v else float("nan")
    hit, miss = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
    fetch = avg("FETCH_SIZE") / 1024  # KB -> MB
    write = avg("WRITE_SIZE") / 1024
    wait = avg("SQ_WAIT_ANY") / max(avg("SQ_WAVE_CYCLES"), 1) * 100
    bw = (fetch * 2 + write) / 1e3 / (us / 1e6) if us else float("nan")  # FETCH_SIZE under-counts 2x on gfx950
    print(f"{k:70s} {us:7.1f} {100 * hit / max(hit + miss, 1):7.1f} {fetch:9.1f} {write:9.1f} {bw:9.1f} {wait:8.1f}")
