"""Diagnostic: what does the lookahead dedup chain (side stream) cost the local step?

Times three variants of the bench's k64 fp32 local step on the same box (not training
benchmarks -- the variants that skip the dedup do not compute a valid plan per step):

  full      the real step: forward + backward of batch t, dedup of batch t+1 / t+2 beside it
  compute   forward + backward only, reading plans precomputed once per pool batch (no side
            stream at all): the compute chain's time without the dedup's competition
  dedup     the dedup chain only (csr_rows + sort + RLE of every batch, back to back)

If ``compute`` is far below ``full``, the side stream's competition for CUs / bandwidth is what
the step pays for the dedup; if ``full`` ~ max(compute, dedup), the chains overlap well.
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
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig, _LocalSlot  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--only", default="", help="'dedup': after the warm-up steps time only the dedup chain "
                    "(for a kernel profile of it alone)")
    a = ap.parse_args()
    K.set_debug_checks(False)
    dev = torch.device("cuda:0")
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn}[a.dtype]
    cfg = FMConfig(vocabulary_size=125_000_000, factor_num=a.k, loss_type="logistic", batch_size=131072,
                   init_value_range=0.01, seed=42, dtype=dtype, opt=K.OptConfig("adagrad", lr=0.01), mode="local")
    m = FactorizationMachine(cfg, device=dev)
    gen = CriteoSynth(cfg.vocabulary_size, seed=1000, device=dev)
    pool = [gen.batch(131072) for _ in range(a.pool)]
    P = len(pool)

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    # full step (bench's call pattern, depth-2 lookahead); --only dedup: 3 steps (the dictionary warms up)
    for i in range(3 if a.only == "dedup" else 6):
        m.train_step(pool[i % P], pool[(i + 1) % P], pool[(i + 2) % P])
    full = (0.0 if a.only == "dedup" else
            timed(lambda i: m.train_step(pool[i % P], pool[(i + 1) % P], pool[(i + 2) % P]), a.steps))
    # precomputed plans, one slot per pool batch
    m.ws.ensure(pool[0].B, max(b.nnz for b in pool))
    slots = [_LocalSlot() for _ in range(P)]
    if a.only == "dedup":
        dedup = timed(lambda i: m._plan_into(slots[i % P], pool[i % P]), a.steps)
        print(f"[side_chain] k={a.k} {a.dtype}: full {full:.3f} ms/step, dedup-only {dedup:.3f}", flush=True)
        m.close()
        return 0
    plans = [m._plan_into(slots[j], pool[j]) for j in range(P)]
    torch.cuda.synchronize()
    compute = timed(lambda i: m._fwd_bwd_local(pool[i % P], *plans[i % P]), a.steps)
    dedup = timed(lambda i: m._plan_into(slots[i % P], pool[i % P]), a.steps)
    print(f"[side_chain] k={a.k} {a.dtype}: full {full:.3f} ms/step, compute-only {compute:.3f}, "
          f"dedup-only {dedup:.3f}", flush=True)
    m.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
