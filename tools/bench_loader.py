#!/usr/bin/env python3
"""Host-only timing of the native text loader (csrc/cpu/loader.cpp), per epoch: raw mode (line
bytes for the GPU tokenizer), parse mode (CPU parser -> CSR) and binary mode (.fmb caches -> CSR
assembly, data/bincache.py), with weight files, on the e2e
tool's shape (Criteo-shaped libsvm lines, vocabulary 800k, batch 50000).  Runs without a GPU.

usage: python tools/bench_loader.py [--lines 250000] [--files 4] [--epochs 3] [--threads 8]
"""

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_tffm_amd.data.synthetic import write_libsvm  # noqa: E402
from fast_tffm_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=250_000)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--batch", type=int, default=50_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--modes", default="raw,parse", help="comma list of raw, parse, binary")
    ap.add_argument("--no-weights", action="store_true")
    ap.add_argument("--dir", default="/tmp/fm_loader_bench")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    files, wfiles = [], []
    for i in range(a.files):
        p, w = os.path.join(a.dir, f"train_{i}"), os.path.join(a.dir, f"weight_{i}")
        if not os.path.exists(p) or not os.path.exists(w):
            write_libsvm(p, a.lines, shape="criteo", vocab_size=800_000, seed=i, weights_path=w)
        files.append(p)
        wfiles.append(w)
    nbytes = sum(os.path.getsize(f) for f in files)
    print(f"{a.files} files x {a.lines} lines, {nbytes / a.files / a.lines:.0f} B/line, batch {a.batch}, "
          f"{a.threads} threads", flush=True)
    import numpy as np

    B = a.batch
    nb = int(B * nbytes / a.files / a.lines * 1.5) + 4096
    bufs = [(np.empty(nb, np.uint8), np.empty(B + 1, np.int64), np.empty(B, np.float32)) for _ in range(8)]
    slots = [[b.ctypes.data, b.size, ls.ctypes.data, ls.size, w.ctypes.data, w.size] for b, ls, w in bufs]
    bfiles = []
    if "binary" in a.modes:
        from fast_tffm_amd.data.bincache import convert_files

        bfiles = [pth for pth, _ in convert_files(files, None if a.no_weights else wfiles,
                                                   os.path.join(a.dir, "fmb"), 800_000, threads=a.threads)]
    for mode in a.modes.split(","):
        binary = mode == "binary"
        L = native.cpu().TextLoader(raw_slots=slots if mode == "raw" else [], files=bfiles if binary else files,
                                    weight_files=[] if a.no_weights or binary else wfiles, batch_size=a.batch,
                                    vocab_size=800_000, hash_feature_id=False, shuffle=True, num_epochs=a.epochs,
                                    seed=1, threads=a.threads, rank=0, world=1, queue_size=4, start_epoch=0,
                                    skip_batches=0, raw=mode == "raw", binary=binary, rows=False)
        t = time.time()
        per_epoch, n, cur = [], 0, 0
        while True:
            item = L.next()
            if item is None:
                break
            ep = int(item[-2])
            if ep != cur:
                per_epoch.append((n, time.time() - t))
                t, n, cur = time.time(), 0, ep
            if mode == "raw":
                n += int(item[2])
                L.release(int(item[0]))
            else:
                n += len(item[0])
        per_epoch.append((n, time.time() - t))
        L.close()
        rates = " ".join(f"{k / dt / 1e6:.2f}" for k, dt in per_epoch)
        print(f"[loader {mode}] M ex/s per epoch: {rates}", flush=True)


if __name__ == "__main__":
    main()
