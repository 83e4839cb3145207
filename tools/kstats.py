#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (or the -d directory holding one): per-kernel time per
step (calls/step inferred)."""
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):  # a rocprofv3 -d directory: its kernel_stats.csv, wherever it was written
    found = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
    if not found:
        sys.exit(f"no kernel_stats.csv under {path}")
    path = found[0]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"{'us/step':>9} {'calls':>6} {'avg_us':>9}  kernel   (per-step = total / {steps})")
for r in rows[:30]:
    tot = float(r["TotalDurationNs"]) / 1e3
    print(f"{tot / steps:9.1f} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:120]}")
