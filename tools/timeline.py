#!/usr/bin/env python3
"""Print the kernel timeline of the last full step from a rocprofv3 kernel_trace.csv.

usage: timeline.py run_kernel_trace.csv <kernel-name-substring marking one per step>
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "fm_fwd_kernel"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
if len(idx) < 3:
    sys.exit("not enough steps in trace")
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["Start_Timestamp"])
qcol = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
step_us = (int(rows[b]["Start_Timestamp"]) - t0) / 1000
print(f"{'start_us':>9} {'dur_us':>8} {'q':>3}  kernel   (step = {step_us:.1f} us)")
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r[qcol] if qcol else "-"
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} {q:>3}  {r['Kernel_Name'][:100]}")
