#!/usr/bin/env python3
"""Merge rocprofv3 --pmc counter CSVs (one dir per pass, p1 p2 ...) into a per-kernel table.

Values are averaged per dispatch.  Normalisation (no fudge factors):
  * GRBM_GUI_ACTIVE arrives summed over its instances; the instance count is inferred from
    GRBM / (duration x 2.4 GHz) as the nearest of 1 / 8 / 32 (``inst`` column) and busy
    percentages use the per-instance cycle count, as rocprof's own derived metrics do
    (counter_defs.yaml: VALUBusy, MfmaUtil use reduce(GRBM_GUI_ACTIVE, max)).
  * FETCH_MB is the raw FETCH_SIZE (L2 -> fabric read requests x 64 B, Infinity-Cache hits
    included): it is NOT HBM traffic.  MI355X_MICROARCH.md (HBM section) measured it at exactly
    half the bytes of a wide (16 B / lane) streaming read; ``fetch_x2`` shows that calibrated
    reading separately so either interpretation can be checked.  DRAM_MB counts the L2 read
    requests whose target is DRAM (TCC_EA0_RDREQ_DRAM x 64 B, same caveat on request size).
  * vmem_lat: SQ_INST_LEVEL_VMEM / VMEM instructions (Little's law: cycles a VMEM instruction
    is in flight, issue to data return, averaged);
  * TLB: TCP_UTCL1 translation miss rate; lat = TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ
    (cycles from an L1 miss to the L2 answer, averaged over requests).
"""
import collections
import csv
import glob
import math
import os
import sys

CU_NUM, SIMD_NUM, CLK_MHZ = 256, 1024, 2400.0

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)


def key_of(name: str) -> str | None:
    if not name.startswith(("void fm::", "fm::", "void rocprim")):
        return None
    return name.split("(")[0].replace("void ", "")[:58]


for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = key_of(r.get("Kernel_Name", r.get("Kernel-Name", "?")))
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = key_of(r.get("Kernel_Name", "?"))
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def fmt(v, w=7, p=1):
    return f"{v:{w}.{p}f}" if v == v else " " * (w - 3) + "  -"


cols = ["us", "inst", "VALU%", "MFMA%", "VMEMrd/w", "vmem_lat", "L2hit%", "FETCH_MB", "fetch_x2", "DRAM_MB", "WRITE_MB",
        "TLBmiss%", "lat_cyc", "TAbusy%", "wait%", "VALUi/w", "LDSbc/i"]
print(f"{'kernel':58s} " + " ".join(f"{c:>8s}" for c in cols))
for k, c in sorted(acc.items(), key=lambda kv: -sum(dur.get(kv[0], [0]))):
    d = sorted(dur.get(k, [0]))
    us = d[len(d) // 2] if d else 0.0

    def avg(n):
        v = c.get(n)
        return sum(v) / len(v) if v else float("nan")

    gui = avg("GRBM_GUI_ACTIVE")
    inst = float("nan")
    if gui == gui and us > 0:
        r = gui / (us * CLK_MHZ)
        inst = min((1, 8, 32), key=lambda n: abs(math.log(max(r, 1e-9)) - math.log(n)))
    cyc = gui / inst if inst == inst else us * CLK_MHZ  # per-instance active cycles
    valu = 100 * avg("SQ_ACTIVE_INST_VALU") / CU_NUM / cyc
    mfma = 100 * avg("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * SIMD_NUM)
    vmem = avg("SQ_INSTS_VMEM_RD") / max(avg("SQ_WAVES"), 1)
    # Little's law: in-flight VMEM instructions summed per cycle / instructions = cycles each
    vlat = avg("SQ_INST_LEVEL_VMEM") / max(avg("SQ_INSTS_VMEM"), 1)
    hit, miss = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
    l2 = 100 * hit / (hit + miss) if hit == hit and miss == miss and hit + miss > 0 else float("nan")
    fetch = avg("FETCH_SIZE") / 1024
    dram = avg("TCC_EA0_RDREQ_DRAM_sum") * 64 / 2**20
    write = avg("WRITE_SIZE") / 1024
    th, tm = avg("TCP_UTCL1_TRANSLATION_HIT"), avg("TCP_UTCL1_TRANSLATION_MISS")
    tlb = 100 * tm / (th + tm) if th == th and tm == tm and th + tm > 0 else float("nan")
    lat = avg("TCP_TCC_READ_REQ_LATENCY") / max(avg("TCP_TCC_READ_REQ"), 1)
    ta = 100 * avg("TA_TA_BUSY") / (cyc * CU_NUM)
    wait = 100 * avg("SQ_WAIT_ANY") / max(avg("SQ_WAVE_CYCLES"), 1)
    valu_i = avg("SQ_INSTS_VALU") / max(avg("SQ_WAVES"), 1)          # VALU instructions per wave
    ldsbc = avg("SQ_LDS_BANK_CONFLICT") / max(avg("SQ_INSTS_LDS"), 1)  # conflict cycles per LDS instruction
    vals = [us, inst, valu, mfma, vmem, vlat, l2, fetch, 2 * fetch, dram, write, tlb, lat, ta, wait, valu_i, ldsbc]
    print(f"{k:58s} " + " ".join(fmt(v, 8) for v in vals))
