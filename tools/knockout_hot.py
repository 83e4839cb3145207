"""Knockout experiment: how much of the step do the batch's hottest rows cost?

Builds the bench's Criteo-shaped batches, removes every occurrence of the batch's `--drop`
most frequent ids (examples keep their remaining features), and times the training step on
the result.  Run once with --drop 0 and once with --drop N under `rocprofv3 --kernel-trace
--stats` to see how the forward / chunk-backward kernel times depend on the hot occurrences
(the work a dense-row MFMA path would take over).  Not a valid training benchmark: the
knocked-out batches are a different workload.
"""

from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fast_tffm_amd.data.batch import Batch  # noqa: E402
from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402


def knock(b: Batch, drop: int) -> Batch:
    if drop <= 0:
        return b
    ids = b.ids.long()
    u, c = torch.unique(ids, return_counts=True)
    hot = u[torch.argsort(c, descending=True)[:drop]]
    keep = ~torch.isin(ids, hot)
    B = b.B
    ex = torch.repeat_interleave(torch.arange(B, device=ids.device), b.offsets[1:] - b.offsets[:-1])
    per = torch.bincount(ex[keep], minlength=B)
    off = torch.zeros(B + 1, dtype=torch.int32, device=ids.device)
    off[1:] = torch.cumsum(per, 0).to(torch.int32)
    nid = b.ids[keep].contiguous()
    return Batch(labels=b.labels, offsets=off, ids=nid, vals=None, weights=None, nnz=int(nid.numel()),
                 max_feats=b.max_feats, offsets_host=off.cpu())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--drop", type=int, default=0)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--k", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn}[a.dtype]
    cfg = FMConfig(vocabulary_size=125_000_000, factor_num=a.k, loss_type="logistic", batch_size=131072,
                   init_value_range=0.01, seed=42, dtype=dtype, opt=K.OptConfig("adagrad", lr=0.01),
                   mode="local")
    model = FactorizationMachine(cfg, device=dev)
    gen = CriteoSynth(cfg.vocabulary_size, seed=1000, device=dev)
    pool = [knock(gen.batch(131072), a.drop) for _ in range(a.pool)]
    torch.cuda.synchronize()
    for i in range(5):
        model.train_step(pool[i % a.pool], pool[(i + 1) % a.pool])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        model.train_step(pool[i % a.pool], pool[(i + 1) % a.pool])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"[knockout] drop={a.drop} nnz={pool[0].nnz} ms/step={ms:.3f}", flush=True)
    model.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
