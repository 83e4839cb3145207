#!/usr/bin/env python3
"""Input-pipeline throughput: text lines/s of the Python reader, the native C++
loader (CPU parser), the native loader + GPU tokenizer, and the native loader
over binary CSR caches (.fmb, converted once), on Criteo-shaped libsvm files
written to a scratch directory.

usage: python tools/bench_input.py [--lines N] [--files F] [--batch B] [--threads T] [--dir D]
"""

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fast_tffm_amd.data import bincache  # noqa: E402
from fast_tffm_amd.data.reader import NativeTextReader, TextBatchReader  # noqa: E402
from fast_tffm_amd.data.synthetic import write_libsvm  # noqa: E402


def run(reader):
    t = time.time()
    n = nnz = 0
    for b in reader:
        n += b.B
        nnz += b.nnz
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return n, nnz, time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=200_000, help="lines per file")
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--batch", type=int, default=50_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--dir", default="/tmp/fm_input_bench")
    ap.add_argument("--skip-python", action="store_true")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    files, wfiles = [], []
    t = time.time()
    for i in range(a.files):
        p, w = os.path.join(a.dir, f"train_{i}"), os.path.join(a.dir, f"weight_{i}")
        if not os.path.exists(p):
            write_libsvm(p, a.lines, shape="criteo", vocab_size=1_000_000, seed=i, weights_path=w)
        files.append(p)
        wfiles.append(w)
    mb = sum(os.path.getsize(f) for f in files) / 1e6
    print(f"data: {a.files} x {a.lines} lines, {mb:.0f} MB (written in {time.time() - t:.1f}s)", flush=True)
    kw = dict(vocab_size=1_000_000, num_epochs=2, seed=1, parse_threads=a.threads)
    results = {}
    if not a.skip_python:
        results["python reader"] = run(TextBatchReader(files, wfiles, a.batch, **kw))
    results["native loader (CPU parse)"] = run(NativeTextReader(files, wfiles, a.batch, **kw))
    if torch.cuda.is_available():
        run(NativeTextReader(files[:1], wfiles[:1], a.batch, gpu_parse="cuda", **dict(kw, num_epochs=1)))  # warm-up
        results["native loader + GPU tokenizer"] = run(NativeTextReader(files, wfiles, a.batch, gpu_parse="cuda",
                                                                        **kw))
    t = time.time()
    caches = [p for p, _ in bincache.convert_files(files, wfiles, os.path.join(a.dir, "fmb"), 1_000_000,
                                                   threads=a.threads)]
    print(f"converted to .fmb in {time.time() - t:.1f}s", flush=True)
    results["native loader (.fmb cache)"] = run(NativeTextReader(caches, None, a.batch, **kw))
    for k, (n, nnz, dt) in results.items():
        print(f"{k:32s} {n / dt / 1e6:7.2f} M lines/s  {nnz / dt / 1e6:8.1f} M features/s  ({n} lines, {dt:.2f}s)",
              flush=True)


if __name__ == "__main__":
    main()
