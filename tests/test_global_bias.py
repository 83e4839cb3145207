"""Optional global bias b0 (model extension; the reference scorer has none,
cc/fm_scorer_op.h:134-136): pred += b0, dL/db0 = sum_i dpred_i, updated with the
table's optimizer; multi-rank runs all-reduce the gradient so every rank holds the
same b0."""

import os

import torch
import torch.multiprocessing as mp

from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

from oracle import fm_scores

V, KF = 500, 8


def _cfg(mode="local", bcfg=64, opt="adagrad"):
    return FMConfig(vocabulary_size=V, factor_num=KF, loss_type="logistic", batch_size=bcfg, init_value_range=0.1,
                    seed=3, mode=mode, grad_reduce="mean", opt=K.OptConfig(opt, lr=0.1, initial_accumulator=0.1),
                    global_bias=True, threads=1)


def test_bias_gradient_and_adagrad_update():
    m = FactorizationMachine(_cfg(), device="cpu")
    b = random_batch(64, V, max_feats=6, seed=4)
    p0 = m.table.reference_rows().double()
    m.train_step(b)
    pred, _, _ = fm_scores(p0, b.offsets, b.ids, b.vals)
    y, wt = b.labels.double(), b.weights.double()
    g = float((wt * (torch.sigmoid(pred) - y)).mean())
    acc = 0.1 + g * g
    torch.testing.assert_close(m.gbias.double(), torch.tensor([-0.1 * g / acc ** 0.5], dtype=torch.float64),
                               rtol=1e-5, atol=1e-7)
    # the forward uses it
    out = m.predict(b)
    ref, _, _ = fm_scores(m.table.reference_rows().double(), b.offsets, b.ids, b.vals)
    torch.testing.assert_close(out.double(), ref + float(m.gbias), rtol=1e-5, atol=1e-6)


def _free_port():
    from ports import free_port

    return free_port()


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cpu")
    m = FactorizationMachine(_cfg("shard", 32 * world), device="cpu", dist=ctx)
    for s in range(3):
        m.train_step(random_batch(32, V, max_feats=6, seed=100 * s + rank))
    torch.save({"b": m.gbias.clone(), "acc": m.gbias_s0.clone()}, os.path.join(out, f"r{rank}.pt"))
    fmdist.shutdown()


def test_bias_all_reduced_across_ranks_equals_single_process(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(os.path.join(tmp_path, f"r{i}.pt"), weights_only=True) for i in range(2)]
    assert torch.equal(r[0]["b"], r[1]["b"])
    from test_distributed import _concat

    single = FactorizationMachine(_cfg("local", 64), device="cpu")
    for s in range(3):
        single.train_step(_concat([random_batch(32, V, max_feats=6, seed=100 * s + k) for k in range(2)]))
    torch.testing.assert_close(r[0]["b"], single.gbias, rtol=1e-5, atol=1e-7)
