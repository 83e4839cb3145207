"""Dedup chain alone (csr_rows codes + grouping + chunk plan) on Criteo-shaped batches, per method.

Times K.dedup back to back on a pool of batches (no step beside it), once per sort backend named in
``--algo`` (rocprim = onesweep, fm = in-tree radix sort).  Run under ``rocprofv3 --kernel-trace
--stats`` for per-kernel times.

    python tools/bench_dedup.py [--algo rocprim,fm] [--iters 30] [--vocab 125000000]
"""

from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="rocprim,fm", help="comma list of sort backends (rocprim, fm)")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--vocab", type=int, default=125_000_000)
    a = ap.parse_args()
    K.set_debug_checks(False)
    dev = torch.device("cuda:0")
    gen = CriteoSynth(a.vocab, seed=1000, device=dev)
    kb = max(1, (a.vocab - 1).bit_length())
    pool = []
    for _ in range(a.pool):
        b = gen.batch(131072)
        sb = K.slot_bits_for(b.B, b.max_feats)
        pool.append((b.ids.to(torch.int32), b.offsets, b.nnz, sb))
    for algo in a.algo.split(","):
        K.set_sort_algo(algo)
        ws = K.DedupWorkspace(max(p[0].numel() for p in pool), dev, 32)

        def run(i):
            ids, off, nnz, sb = pool[i % len(pool)]
            codes = K.csr_rows(off, out=ws.ex_of_occ[:nnz], nnz=nnz, slot_bits=sb)
            K.dedup(ids, ws=ws, key_bits=kb, ex_of_occ=codes, ex_shift=sb, offsets=off)

        for i in range(3):
            run(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.iters):
            run(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.iters * 1e3
        n = sum(p[2] for p in pool) / len(pool)
        print(f"[bench_dedup] {algo:8s} n={n / 1e6:.2f}M: {ms:.3f} ms per dedup (csr_rows + grouping + plan)",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
