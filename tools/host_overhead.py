#!/usr/bin/env python3
"""Host-side cost of one training step: wall time of the Python train_step calls
alone (no device sync inside the loop) vs device time per step.  If the two are
close, the step is launch/host-bound.

usage: python tools/host_overhead.py [--mode shard] [--steps 30]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402
from fast_tffm_amd.parallel import dist as fmdist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="shard")
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--batch", type=int, default=131072)
ap.add_argument("--vocab", type=int, default=125_000_000)
ap.add_argument("--prefetch-rows", default="auto", choices=["auto", "on", "off"])
ap.add_argument("--overlap-grads", default="auto", choices=["auto", "on", "off"])
ap.add_argument("--depth", type=int, default=2, help="batches of lookahead passed to train_step (1 or 2)")
a = ap.parse_args()
ctx = fmdist.init_distributed(force_pg=a.mode != "local")
cfg = FMConfig(vocabulary_size=a.vocab, factor_num=64, loss_type="logistic", batch_size=a.batch, seed=1,
               opt=K.OptConfig("adagrad", lr=0.01), mode=a.mode, prefetch_rows=a.prefetch_rows,
               overlap_grads=a.overlap_grads)
m = FactorizationMachine(cfg, device=ctx.device, dist=ctx if a.mode != "local" else None)
gen = CriteoSynth(a.vocab, seed=3, device=ctx.device)
pool = [gen.batch(a.batch) for _ in range(4)]


def step(i):
    return m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4] if a.depth > 1 else None)


for i in range(5):
    step(i)
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for i in range(5, 5 + a.steps):  # (the batch order continues: the executor planned ahead for it)
    h0 = time.perf_counter()
    step(i)
    host.append(time.perf_counter() - h0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / a.steps
host.sort()
print(f"mode={a.mode} wall/step={wall * 1e3:.3f} ms  host call/step median={host[len(host) // 2] * 1e3:.3f} ms "
      f"min={host[0] * 1e3:.3f} max={host[-1] * 1e3:.3f}")
# pure Python overhead: the same calls under the profiler's CPU view
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU]) as prof:
    for i in range(5 + a.steps, 10 + a.steps):
        step(i)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
fmdist.shutdown()
