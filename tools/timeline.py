#!/usr/bin/env python3
"""Print the kernel timeline of the last full step from a rocprofv3 kernel_trace.csv.

usage: timeline.py run_kernel_trace.csv <kernel-name-substring marking one per step> [run_memory_copy_trace.csv]

With a memory-copy trace, the step's copies are listed too (direction and bytes), so a blit kernel
(``__amd_rocclr_copyBuffer``) can be told apart as a device copy or a host transfer.
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
t1 = int(rows[b]["Start_Timestamp"])
qcol = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
step_us = (t1 - t0) / 1000
events = []
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r[qcol] if qcol else "-"
    events.append((s, e, q, r["Kernel_Name"][:100]))
if len(sys.argv) > 3:
    for r in csv.DictReader(open(sys.argv[3])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            kind = r.get("Direction") or r.get("Kind") or r.get("Operation") or "copy"
            nb = r.get("Bytes") or r.get("Size") or "?"
            events.append((s, e, "mem", f"[memcpy {kind} {nb} B]"))
events.sort()
print(f"{'start_us':>9} {'dur_us':>8} {'q':>3}  kernel   (step = {step_us:.1f} us)")
for s, e, q, name in events:
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} {q:>3}  {name}")
