"""Bounded staleness trains as well as the synchronous step (round-5 verdict, item 2).

The planted-teacher task of tests/test_precision_parity_gpu.py (a k=8 FM teacher over 24 Zipf fields
labels Criteo-shaped examples): 4 ranks on one GPU (gloo + the asynchronous relay, tests/relay.py) train
the row-sharded table for 400 steps with ``staleness = 1`` -- every step reads the table one step
stale and applies its gradient one step late, as the reference's asynchronous parameter-server
workers do (run_tffm.py:204-211) -- on 1024 examples each of the same global batches a synchronous
single process trains on (the synchronous W-rank step equals it: tests/test_distributed.py,
tests/test_dist_gpu_relay.py).  The held-out logloss must agree within 0.5% (relative), and both
must clearly beat the label prior.
"""

import math
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

V, B, STEPS, NTRAIN, NHELD, W = 50_000, 4096, 400, 48, 8, 4
FIELDS = [12, 40, 100, 300, 800, 2000, 5000, 9000] * 3


def _data(dev):
    from fast_tffm_amd.data.batch import Batch
    from fast_tffm_amd.data.synthetic import CriteoSynth

    g = torch.Generator(device=dev).manual_seed(77)
    w = torch.randn(V, generator=g, device=dev) * 0.6
    v = torch.randn(V, 8, generator=g, device=dev) * 0.35
    synth = CriteoSynth(V, fields=FIELDS, alpha=1.05, seed=99, device=dev)
    out = []
    for _ in range(NTRAIN + NHELD):
        b = synth.batch(B)
        ids = b.ids.long().view(B, len(FIELDS))
        s1 = v[ids].sum(1)
        score = w[ids].sum(1) + 0.5 * (s1.pow(2) - v[ids].pow(2).sum(1)).sum(1) - 1.0
        labels = (torch.rand(B, generator=g, device=dev) < torch.sigmoid(score)).float()
        out.append(Batch(labels, b.offsets, b.ids, None, None, b.nnz, max_feats=b.max_feats))
    return out[:NTRAIN], out[NTRAIN:]


def _slice(b, r, n):
    """Examples [r n, (r + 1) n) of a batch whose examples all have len(FIELDS) features."""
    from fast_tffm_amd.data.batch import Batch

    F = len(FIELDS)
    offs = torch.arange(n + 1, dtype=torch.int32, device=b.ids.device) * F
    return Batch(b.labels[r * n:(r + 1) * n].contiguous(), offs, b.ids[r * n * F:(r + 1) * n * F].contiguous(),
                 None, None, n * F, max_feats=F)


def _cfg(mode, bcfg, staleness=0):
    from fast_tffm_amd.models.fm import FMConfig
    from fast_tffm_amd.ops import kernels as K

    return FMConfig(vocabulary_size=V, factor_num=16, loss_type="logistic", batch_size=bcfg, init_value_range=0.01,
                    seed=5, opt=K.OptConfig("adagrad", lr=0.3), mode=mode, grad_reduce="mean", staleness=staleness)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import relay

    relay.install()
    from fast_tffm_amd.models.fm import FactorizationMachine
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cuda:0")
    train, held = _data(torch.device("cuda:0"))
    n = B // world
    mine = [_slice(b, rank, n) for b in train]
    m = FactorizationMachine(_cfg("shard", n, staleness=1), device="cuda:0", dist=ctx)
    for i in range(STEPS):
        m.train_step(mine[i % NTRAIN], mine[(i + 1) % NTRAIN], mine[(i + 2) % NTRAIN])
    m.flush()
    loss = sum(m.eval_loss(_slice(b, rank, n)) for b in held) / len(held)  # (this rank's quarter)
    torch.save({"loss": loss, "early": m._exchange.early_steps}, os.path.join(out_dir, f"rank{rank}.pt"))
    fmdist.shutdown()


def test_stale_world4_matches_synchronous_heldout_logloss(tmp_path):
    from ports import free_port

    from fast_tffm_amd.models.fm import FactorizationMachine

    mp.spawn(_worker, args=(W, free_port(), str(tmp_path)), nprocs=W, join=True)
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(W)]
    assert all(r["early"] == STEPS - 1 for r in res)
    stale = sum(r["loss"] for r in res) / W  # (equal quarters: the mean over the held-out examples)
    train, held = _data(torch.device("cuda:0"))
    m = FactorizationMachine(_cfg("local", B), device="cuda:0")
    for i in range(STEPS):
        m.train_step(train[i % NTRAIN], train[(i + 1) % NTRAIN])
    sync = sum(m.eval_loss(b) for b in held) / len(held)
    m.close()
    p = sum(float(b.labels.mean()) for b in held) / len(held)
    prior = -(p * math.log(p) + (1 - p) * math.log(1 - p))
    print(f"[staleness parity] W={W} staleness 1: held-out logloss {stale:.5f} vs synchronous {sync:.5f} "
          f"(rel {(stale - sync) / sync:+.2e}; prior {prior:.5f})")
    assert sync < 0.95 * prior and stale < 0.95 * prior, (sync, stale, prior)
    assert abs(stale - sync) / sync < 5e-3, (stale, sync)
