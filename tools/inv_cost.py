"""Cost of the sharded dedup's inverse map (occurrence -> segment scatter) on the local step.

The row-sharded forward reads wire rows through the dedup's inverse map, a scatter of one
4-byte segment id per occurrence (5.1M random writes per Criteo-shaped batch).  The local step
does not need it; this tool times the local k64 step with and without forcing the inverse map
(and the packed occurrence codes the sharded plan uses) into its dedup, to price the scatter.
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
from fast_tffm_amd.models import fm as fm_mod  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--inv", type=int, default=0)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    if a.inv:
        orig = K.dedup

        def dedup_inv(*args, **kw):
            kw["want_inv"] = True
            return orig(*args, **kw)

        fm_mod.K.dedup = dedup_inv
        orig_sb = FactorizationMachine._slot_bits
        FactorizationMachine._slot_bits = staticmethod(lambda b, always=False: orig_sb(b, always=True))
    dev = torch.device("cuda:0")
    cfg = FMConfig(vocabulary_size=125_000_000, factor_num=64, loss_type="logistic", batch_size=131072,
                   init_value_range=0.01, seed=42, opt=K.OptConfig("adagrad", lr=0.01), mode="local")
    m = FactorizationMachine(cfg, device=dev)
    gen = CriteoSynth(cfg.vocabulary_size, seed=1000, device=dev)
    pool = [gen.batch(131072) for _ in range(8)]
    for i in range(5):
        m.train_step(pool[i % 8], pool[(i + 1) % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        m.train_step(pool[i % 8], pool[(i + 1) % 8])
    torch.cuda.synchronize()
    print(f"[inv_cost] inv={a.inv} ms/step={(time.perf_counter() - t0) / a.steps * 1e3:.3f}", flush=True)
    m.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
