"""Random-row gather rates on the bench's table (125M x 64 fp32 rows + w), the anchor for the
step's roofline: what the memory system delivers for the access patterns the forward and the
chunk backward are made of, measured alone.

  batch rows    the 5.1M row reads of a Criteo-shaped batch (hot rows repeat: L2 hits), as the
                forward issues them
  unique rows   the batch's ~378k distinct rows once each (the backward's table rows)
  random rows   the same number of uniformly random rows of the whole table

Kernel: K.gather_rows (hip/shard.hip gather_rows_kernel: one 256-B row per 16-lane group, w with
it, [v | w | 0 0 0] fp32 rows written out).  Reported: rows/s and GB/s of row bytes read (256 B + the
w word's 64-B sector counted as 4 B logical).
"""

from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    K.set_debug_checks(False)
    dev = torch.device("cuda:0")
    V, Kp = 125_000_000, 64
    v = torch.empty((V, Kp), dtype=torch.float32, device=dev)
    v.uniform_(-0.01, 0.01)
    w = torch.zeros(V, dtype=torch.float32, device=dev)
    table = K.TableState(v=v, w=w)
    b = CriteoSynth(V, seed=1000, device=dev).batch(131072)
    rows = b.ids.to(torch.int32)
    uniq = torch.unique(rows).to(torch.int32)
    rnd = torch.randint(0, V, (uniq.numel(),), device=dev, dtype=torch.int64).to(torch.int32)
    cases = [("batch rows", rows), ("unique rows", uniq), ("random rows", rnd),
             ("unique rows, shuffled", uniq[torch.randperm(uniq.numel(), device=dev)])]
    for name, req in cases:
        out = torch.empty((req.numel(), Kp + 4), dtype=torch.float32, device=dev)
        for _ in range(3):
            K.gather_rows(req, table, Kp, out)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            K.gather_rows(req, table, Kp, out)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / n * 1e6
        R = req.numel()
        print(f"[gather_roofline] {name:22s} R={R / 1e6:6.3f}M  {us:8.1f} us  {R / us:7.1f} Mrows/s  "
              f"{R * (Kp * 4 + 4) / us / 1e6:6.2f} TB/s read", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
