#!/usr/bin/env python3
"""Host-side profile of the row-sharded executor's steady-state steps (cProfile over train_step calls,
no device sync inside the loop), RCCL world 1, the N > 1 compute path (FM_SHARD_W1_LOCAL=0 unless
--local-w1).  Prints the executor's host time per step (wall minus the blocked waits of
ShardExchange._await) and the functions with the most own / cumulative time.

usage: python tools/host_profile.py [--steps 40] [--batch 131072] [--staleness 0|1] [--sort tottime]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--batch", type=int, default=131072)
ap.add_argument("--vocab", type=int, default=125_000_000)
ap.add_argument("--staleness", type=int, default=0)
ap.add_argument("--local-w1", action="store_true")
ap.add_argument("--sort", default="tottime")
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
if not a.local_w1:
    os.environ["FM_SHARD_W1_LOCAL"] = "0"

from fast_tffm_amd.parallel import dist as fmdist  # noqa: E402

fmdist.ensure_hw_queues()
import torch  # noqa: E402

from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
ctx = fmdist.init_distributed(force_pg=True)
cfg = FMConfig(vocabulary_size=a.vocab, factor_num=64, loss_type="logistic", batch_size=a.batch, seed=1, mode="shard",
               opt=K.OptConfig("adagrad", lr=0.01), staleness=a.staleness)
m = FactorizationMachine(cfg, device=ctx.device, dist=ctx)
gen = CriteoSynth(a.vocab, seed=3, device=ctx.device)
pool = [gen.batch(a.batch) for _ in range(4)]
ex = m._exchange


def step(i):
    return m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])


for i in range(8):
    step(i)
torch.cuda.synchronize()
w0 = ex.host_wait_s
prof = cProfile.Profile()
t0 = time.perf_counter()
prof.enable()
for i in range(8, 8 + a.steps):
    step(i)
prof.disable()
wall = time.perf_counter() - t0
torch.cuda.synchronize()
dev = (time.perf_counter() - t0) / a.steps
waited = ex.host_wait_s - w0
print(f"[host_profile] staleness={a.staleness} local_w1={ex.local_w1}: "
      f"host {(wall - waited) / a.steps * 1e6:.0f} us/step "
      f"(wall {wall / a.steps * 1e6:.0f}, blocked {waited / a.steps * 1e6:.0f}; cProfile overhead included), "
      f"device-bound step {dev * 1e3:.3f} ms")
pstats.Stats(prof).sort_stats(a.sort).print_stats(a.top)
fmdist.shutdown()
