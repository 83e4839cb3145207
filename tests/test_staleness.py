"""Bounded-staleness row-sharded steps (``staleness = 1``) on CPU (gloo).

The reference trains asynchronously (between-graph replication, no SyncReplicasOptimizer:
run_tffm.py:204-211, fm_model.py:345-348): workers read whatever the parameter servers hold and push
gradients without waiting.  ``ShardExchange`` with ``staleness = 1`` is the deterministic form: step t
reads every row with the merged gradients of steps <= t-2 applied, and the gradient of step t-1 is
applied (by the rows' owners) while step t computes.  So

* one rank equals an fp64 oracle that applies each step's gradient one step late (Adagrad);
* W ranks equal one rank on the concatenated batches (grad_reduce = mean), at W = 2 / 4 / 8, with
  and without lookahead batches (with: the rows of step t+1 are gathered and exchanged during step t);
* and the result differs from the synchronous step (it really is stale).
"""

import os

import pytest
import torch
import torch.multiprocessing as mp

from fast_tffm_amd.data.batch import Batch
from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

V, KF, B, STEPS, LR = 997, 8, 24, 5, 0.1


def _free_port() -> int:
    from ports import free_port

    return free_port()


def _cfg(mode, bcfg, staleness):
    return FMConfig(vocabulary_size=V, factor_num=KF, loss_type="logistic", factor_lambda=0.05, bias_lambda=0.02,
                    batch_size=bcfg, init_value_range=0.1, seed=11, mode=mode, grad_reduce="mean",
                    opt=K.OptConfig("adagrad", lr=LR, initial_accumulator=0.1), threads=1, staleness=staleness)


def _batch(step, rank):
    return random_batch(B, V, max_feats=10, seed=1000 * step + rank)


def _concat(batches):
    offs, ids, vals, labels, weights, base = [torch.zeros(1, dtype=torch.int32)], [], [], [], [], 0
    for b in batches:
        offs.append(b.offsets[1:] + base)
        base += b.nnz
        ids.append(b.ids)
        vals.append(b.vals)
        labels.append(b.labels)
        weights.append(b.weights)
    return Batch(torch.cat(labels), torch.cat(offs), torch.cat(ids), torch.cat(vals), torch.cat(weights), base)


def _worker(rank, world, port, out_dir, staleness, lookahead, concat_of):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cpu", force_pg=True)
    # concat_of > 0: one rank training on the concatenation of concat_of ranks' batches
    m = FactorizationMachine(_cfg("shard", 16 * max(1, concat_of), staleness), device="cpu", dist=ctx)  # (mean: / W)
    if concat_of:
        bs = [_concat([_batch(s, r) for r in range(concat_of)]) for s in range(STEPS)]
    else:
        bs = [_batch(s, rank) for s in range(STEPS)]
    losses = []
    for s in range(STEPS):
        nb = bs[s + 1] if lookahead and s + 1 < STEPS else None
        nb2 = bs[s + 2] if lookahead and s + 2 < STEPS else None
        losses.append(m.train_step(bs[s], nb, nb2).mean_loss())
    early = m._exchange.early_steps
    m.flush()
    torch.save({"gids": m.table.global_ids(), "rows": m.table.reference_rows(), "acc": m.table.s0v[:, :KF].clone(),
                "losses": losses, "early": early}, os.path.join(out_dir, f"rank{rank}.pt"))
    fmdist.shutdown()


def _run(tmp_path, world, staleness=1, lookahead=True, concat_of=0):
    d = tmp_path / f"w{world}_s{staleness}_l{int(lookahead)}_c{concat_of}"
    d.mkdir()
    mp.spawn(_worker, args=(world, _free_port(), str(d), staleness, lookahead, concat_of), nprocs=world, join=True)
    return [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def _assemble(res):
    rows = torch.zeros(V, KF + 1, dtype=torch.float32)
    for r in res:
        g = r["gids"]
        ok = g < V
        rows[g[ok]] = r["rows"][ok]
    return rows


def _delayed_oracle():
    """fp64: step t's gradient at the current parameters, then the PREVIOUS step's gradient applied
    (Adagrad on its touched rows); the last gradient applied at the end (the flush)."""
    from oracle import fm_objective, touched_rows

    init = FactorizationMachine(_cfg("local", 16, 0), device="cpu").table.reference_rows().double()
    params, acc = init.clone(), torch.full_like(init, 0.1)
    pending = None
    for s in range(STEPS):
        b = _batch(s, 0)
        p = params.clone().requires_grad_(True)
        obj, _, _ = fm_objective(p, b, "logistic", 0.05, 0.02, 16)
        (g,) = torch.autograd.grad(obj, p)
        cur = (g, touched_rows(b, V))
        if pending is not None:
            gp, tp = pending
            acc[tp] += gp[tp] ** 2
            params[tp] -= LR * gp[tp] / acc[tp].sqrt()
        pending = cur
    gp, tp = pending
    acc[tp] += gp[tp] ** 2
    params[tp] -= LR * gp[tp] / acc[tp].sqrt()
    return params, acc


def test_one_rank_equals_delayed_apply_oracle(tmp_path):
    res = _run(tmp_path, 1)
    assert res[0]["early"] == STEPS - 1  # rows of steps 1.. gathered and exchanged a step ahead
    params, acc = _delayed_oracle()
    torch.testing.assert_close(_assemble(res).double(), params, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(res[0]["acc"][:V].double(), acc[:, 1:], rtol=1e-4, atol=1e-6)
    # without lookahead batches the rows are gathered inside the step: the same semantics
    res_nl = _run(tmp_path, 1, lookahead=False)
    assert res_nl[0]["early"] == 0
    torch.testing.assert_close(_assemble(res_nl), _assemble(res), rtol=0, atol=0)


@pytest.mark.parametrize("world,lookahead", [(2, True), (2, False), (4, True), (8, True)])
def test_ranks_equal_one_rank_on_concatenated_batches(tmp_path, world, lookahead):
    res = _run(tmp_path, world, lookahead=lookahead)
    if lookahead:
        assert all(r["early"] == STEPS - 1 for r in res)
    ref = _run(tmp_path, 1, concat_of=world)
    torch.testing.assert_close(_assemble(res), _assemble(ref), rtol=1e-5, atol=1e-7)
    for s in range(STEPS):  # rank losses average to the single rank's (the same stale parameters)
        got = sum(r["losses"][s] for r in res) / world
        assert abs(got - ref[0]["losses"][s]) < 1e-5


def test_stale_differs_from_synchronous(tmp_path):
    stale = _assemble(_run(tmp_path, 2))
    sync = _assemble(_run(tmp_path, 2, staleness=0))
    assert not torch.allclose(stale, sync, rtol=1e-6, atol=1e-7)
    assert (stale - sync).abs().max() < 0.05  # (one step of delay: close, not equal)
