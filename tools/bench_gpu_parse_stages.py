#!/usr/bin/env python3
"""Stage timing of the GPU-tokenizer input path (native loader in raw mode -> pinned staging
-> H2D + hip/parse.hip), to find which stage caps the file-fed training throughput.

usage: python tools/bench_gpu_parse_stages.py [--lines 250000] [--files 4] [--batch 50000] [--threads 8]
"""

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fast_tffm_amd.data.reader import NativeTextReader  # noqa: E402
from fast_tffm_amd.data.synthetic import write_libsvm  # noqa: E402
from fast_tffm_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=250_000)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--batch", type=int, default=50_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/fm_stage_bench")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    files = []
    for i in range(a.files):
        p = os.path.join(a.dir, f"train_{i}")
        if not os.path.exists(p):
            write_libsvm(p, a.lines, shape="criteo", vocab_size=800_000, seed=i)
        files.append(p)
    n_ex = a.files * a.lines * a.epochs
    args = dict(files=files, weight_files=[], batch_size=a.batch, vocab_size=800_000, hash_feature_id=False,
                shuffle=True, num_epochs=a.epochs, seed=1, threads=a.threads, rank=0, world=1, queue_size=4)
    r = NativeTextReader(files, None, a.batch, vocab_size=800_000, num_epochs=a.epochs, seed=1,
                         parse_threads=a.threads, gpu_parse="cuda")
    # 1) the loader alone: raw batches assembled into the reader's page-locked slots (released at once)
    L = native.cpu().TextLoader(start_epoch=0, skip_batches=0, raw=True, binary=False, rows=False,
                                raw_slots=r._raw_slots(), **args)
    t = time.time()
    nb = 0
    while True:
        item = L.next()
        if item is None:
            break
        if isinstance(item[0], int):
            L.release(item[0])
        nb += 1
    L.close()
    dt = time.time() - t
    print(f"loader raw assembly (pinned slots): {n_ex / dt / 1e6:7.2f} M ex/s ({nb} batches, {dt:.2f}s)", flush=True)
    # 2) the same into heap buffers + the reader's pinned staging copy (the path of a batch that
    #    does not fit a slot)
    L = native.cpu().TextLoader(start_epoch=0, skip_batches=0, raw=True, binary=False, rows=False, **args)
    t = time.time()
    while True:
        item = L.next()
        if item is None:
            break
        r._stage(item[0], item[1])
    L.close()
    dt = time.time() - t
    print(f"heap batches + pinned staging copy: {n_ex / dt / 1e6:7.2f} M ex/s ({dt:.2f}s)", flush=True)
    # 3) the full reader: + H2D + GPU tokenizer (+ one stream sync per batch)
    t = time.time()
    n = 0
    for b in r:
        n += b.B
    torch.cuda.synchronize()
    dt = time.time() - t
    print(f"reader: slots + H2D + GPU tokenizer: {n / dt / 1e6:7.2f} M ex/s ({dt:.2f}s, {r.fallbacks} CPU fallbacks)",
          flush=True)


if __name__ == "__main__":
    main()
