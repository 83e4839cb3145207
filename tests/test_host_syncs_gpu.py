"""Host synchronisation of the row-sharded executor in steady state (round-5 verdict, item 1).

The N > 1 step reads device-produced counts on the host twice per plan: the per-owner id counts (the
all-to-all split sizes) and, with early rows, the dirty-row counts of the patch.  Both are pinned
copies behind events recorded a step earlier, read through ``ShardExchange._await``: a finished event
costs nothing, an unfinished one blocks (``host_blocks``: back-pressure when the host runs more than a
step ahead) and counts as ``starved_waits`` if the compute stream had nothing left to run.

Steady state at RCCL world 1 on the N > 1 compute path (FM_SHARD_W1_LOCAL=0), 20 steps after warm-up:
* no other host synchronisation anywhere in the step (Event / Stream / device synchronize, .item() /
  .tolist() of device tensors) -- monkeypatched counters;
* no starved wait: the host never holds the GPU back;
* the executor's host time per step (wall time of the train_step calls minus the blocked time) is
  printed (profiles/r6/host_sync.txt records the box's numbers).
"""

import os
import time

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

V, B, WARM, STEPS = 10_000_000, 65536, 6, 20


@pytest.fixture(scope="module")
def rccl_ctx():
    from ports import free_port

    from fast_tffm_amd.parallel import dist as fmdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    ctx = fmdist.init_distributed(backend="nccl", rank=0, world=1, device="cuda:0", force_pg=True)
    yield ctx
    fmdist.shutdown()


class _Counters:
    def __init__(self, monkeypatch):
        self.n = {"event_sync": 0, "stream_sync": 0, "device_sync": 0, "item": 0, "tolist": 0}
        ev_sync, st_sync, dev_sync = torch.cuda.Event.synchronize, torch.cuda.Stream.synchronize, torch.cuda.synchronize
        item, tolist = torch.Tensor.item, torch.Tensor.tolist
        c = self.n

        def wrap(key, fn, cuda_only=False):
            def f(*a, **kw):
                if not cuda_only or (a and isinstance(a[0], torch.Tensor) and a[0].is_cuda):
                    c[key] += 1
                return fn(*a, **kw)
            return f

        monkeypatch.setattr(torch.cuda.Event, "synchronize", wrap("event_sync", ev_sync))
        monkeypatch.setattr(torch.cuda.Stream, "synchronize", wrap("stream_sync", st_sync))
        monkeypatch.setattr(torch.cuda, "synchronize", wrap("device_sync", dev_sync))
        monkeypatch.setattr(torch.Tensor, "item", wrap("item", item, True))
        monkeypatch.setattr(torch.Tensor, "tolist", wrap("tolist", tolist, True))

    def reset(self):
        for k in self.n:
            self.n[k] = 0


@pytest.mark.parametrize("variant", ["emit", "early_patch_split", "stale"])
def test_steady_state_has_no_host_sync_on_the_critical_path(rccl_ctx, variant, monkeypatch):
    monkeypatch.setenv("FM_SHARD_W1_LOCAL", "0")
    monkeypatch.setenv("FM_DEBUG_CHECKS", "0")
    was = K.debug_checks()
    K.set_debug_checks(False)
    kw = {}
    if variant == "early_patch_split":  # every row exchanged: early rows + dirty patch + split backward
        monkeypatch.setenv("FM_SELF_ROWS", "0")
        kw = dict(prefetch_rows="on", overlap_grads="on")
    elif variant == "stale":  # bounded staleness: early rows, apply on its own stream
        kw = dict(staleness=1)
    cfg = FMConfig(vocabulary_size=V, factor_num=64, loss_type="logistic", batch_size=B, seed=1, mode="shard",
                   opt=K.OptConfig("adagrad", lr=0.01), **kw)
    m = FactorizationMachine(cfg, device="cuda", dist=rccl_ctx)
    gen = CriteoSynth(V, seed=3, device="cuda")
    pool = [gen.batch(B) for _ in range(4)]
    torch.cuda.synchronize()
    ex = m._exchange

    def step(i):
        return m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])

    for i in range(WARM):
        step(i)
    torch.cuda.synchronize()
    cnt = _Counters(monkeypatch)
    b0, s0, w0 = ex.host_blocks, ex.starved_waits, ex.host_wait_s
    t0 = time.perf_counter()
    for i in range(WARM, WARM + STEPS):
        step(i)
    wall = time.perf_counter() - t0
    calls = dict(cnt.n)
    monkeypatch.undo()
    K.set_debug_checks(was)
    torch.cuda.synchronize()
    blocks, starved, waited = ex.host_blocks - b0, ex.starved_waits - s0, ex.host_wait_s - w0
    host_us = (wall - waited) / STEPS * 1e6
    print(f"[host_syncs] {variant}: {STEPS} steps, blocking waits {blocks} (starved {starved}), "
          f"host time {host_us:.0f} us/step (wall {wall / STEPS * 1e6:.0f}, waiting {waited / STEPS * 1e6:.0f}), "
          f"calls {calls}, early steps {ex.early_steps}")
    # the only synchronisation is _await's, and only when it blocked
    assert calls["event_sync"] == blocks, calls
    assert calls["stream_sync"] == calls["device_sync"] == calls["item"] == calls["tolist"] == 0, calls
    assert starved == 0, (starved, blocks)
    if variant != "emit":
        assert ex.early_steps >= STEPS
    m.close()
