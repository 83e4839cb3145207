"""Multi-rank correctness on CPU (gloo, world_size 2; shard / dp_dense also at 4 and 8): every exchange mode is a
drop-in replacement for the single-process step.

* ``shard`` (row-sharded table, all-to-all lookups/grads), ``dp`` (replicated,
  sparse all-gather) and ``dp_dense`` (replicated, dense all-reduce) with
  ``grad_reduce = mean`` must equal ONE process training on the concatenated
  global batch (batch_size_cfg scaled by the world size);
* ``shard`` with ``grad_reduce = sum`` equals one process whose example weights
  are multiplied by the world size (the summed per-rank mean losses);
* a checkpoint written by 2 shards restores into a 1-process table (re-shard)
  and into the reference vocab_block layout.
"""

import os

import pytest
import torch
import torch.multiprocessing as mp

from fast_tffm_amd.data.batch import Batch
from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K
from fast_tffm_amd.utils import checkpoint as ckpt

V, KF, B, STEPS, WORLD = 997, 8, 24, 3, 2


def _free_port() -> int:
    from ports import free_port

    return free_port()


def _cfg(mode, grad_reduce, bcfg, mb=0):
    return FMConfig(vocabulary_size=V, factor_num=KF, loss_type="logistic", factor_lambda=0.05, bias_lambda=0.02,
                    batch_size=bcfg, init_value_range=0.1, seed=11, mode=mode, grad_reduce=grad_reduce,
                    opt=K.OptConfig("adagrad", lr=0.1, initial_accumulator=0.1), threads=1, microbatches=mb,
                    overlap_grads="on")  # (split backward: the default with one part)


def _batch(step, rank):
    return random_batch(B, V, max_feats=10, seed=1000 * step + rank)


def _worker(rank, world, port, mode, grad_reduce, out_dir, mb=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cpu")
    m = FactorizationMachine(_cfg(mode, grad_reduce, 16, mb), device="cpu", dist=ctx)
    if mode == "shard":
        assert m._exchange.nparts == max(1, mb)
    bs = [_batch(s, rank) for s in range(STEPS)]
    # shard mode also exercises the lookahead plan (next batch's dedup + id exchange built early)
    # (and, with 2 batches of lookahead, the depth-2 pipeline + early row exchange)
    losses = [m.train_step(bs[s], bs[s + 1] if s + 1 < STEPS and mode == "shard" else None,
                           bs[s + 2] if s + 2 < STEPS and mode == "shard" else None).mean_loss()
              for s in range(STEPS)]
    if mode == "shard":  # the early row exchange + patch path ran (lookahead steps 1..); split-gradient
        assert m._exchange.early_steps == (STEPS - 1 if max(1, mb) == 1 else 0)  # exchange with one part
        assert m._exchange.overlap_grads == (max(1, mb) == 1)
    pred = m.predict(_batch(99, rank))
    torch.save({"gids": m.table.global_ids(), "rows": m.table.reference_rows(), "acc": m.table.s0v[:, :KF].clone(),
                "losses": losses, "pred": pred}, os.path.join(out_dir, f"rank{rank}.pt"))
    ckpt.save_checkpoint(m, os.path.join(out_dir, "log"), m.global_step, ctx=ctx)
    fmdist.shutdown()


def _run_world(tmp_path, mode, grad_reduce, mb=0, world=WORLD):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, mode, grad_reduce, str(tmp_path), mb), nprocs=world, join=True)
    return [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def _concat(batches, weight_mult=1.0):
    offs, ids, vals, labels, weights, base = [torch.zeros(1, dtype=torch.int32)], [], [], [], [], 0
    for b in batches:
        offs.append(b.offsets[1:] + base)
        base += b.nnz
        ids.append(b.ids)
        vals.append(b.vals)
        labels.append(b.labels)
        weights.append(b.weights * weight_mult)
    return Batch(torch.cat(labels), torch.cat(offs), torch.cat(ids), torch.cat(vals), torch.cat(weights), base)


def _single(grad_reduce, world=WORLD):
    bcfg = 16 * world if grad_reduce == "mean" else 16
    m = FactorizationMachine(_cfg("local", "sum", bcfg), device="cpu")
    wm = 1.0 if grad_reduce == "mean" else float(world)
    for s in range(STEPS):
        m.train_step(_concat([_batch(s, r) for r in range(world)], wm))
    return m


def _assemble(res):
    rows = torch.zeros(V, KF + 1)
    for r in res:
        g = r["gids"]
        ok = g < V
        rows[g[ok]] = r["rows"][ok]
    return rows


@pytest.mark.parametrize("mode,grad_reduce,mb", [("shard", "mean", 0), ("shard", "sum", 0), ("shard", "mean", 2),
                                                 ("shard", "sum", 3), ("dp", "mean", 0), ("dp_dense", "mean", 0)])
def test_multi_rank_equals_single_process(tmp_path, mode, grad_reduce, mb):
    """shard: one part (default), 2 and 3 micro-batch parts."""
    res = _run_world(tmp_path, mode, grad_reduce, mb)
    ref = _single(grad_reduce)
    ref_rows = ref.table.reference_rows()
    if mode == "shard":
        got = _assemble(res)
        torch.testing.assert_close(got, ref_rows, rtol=1e-5, atol=1e-7)
    else:  # replicated: every rank holds the full, identical table
        for r in res:
            torch.testing.assert_close(r["rows"], ref_rows, rtol=1e-5, atol=1e-7)
        assert torch.equal(res[0]["rows"], res[1]["rows"])
        if mode == "dp_dense":
            _check_dense_checkpoint(tmp_path, ref)
    # predictions of rank r's eval batch match the single model's
    for rank, r in enumerate(res):
        torch.testing.assert_close(r["pred"], ref.predict(_batch(99, rank)), rtol=1e-5, atol=1e-6)

    if mode == "shard" and grad_reduce == "mean" and mb == 0:
        # re-shard: 2-shard checkpoint -> 1-process table
        m1 = FactorizationMachine(_cfg("local", "sum", 16), device="cpu")
        meta = ckpt.restore_checkpoint(m1, ckpt.latest_checkpoint(str(tmp_path / "log")))
        assert meta["shard_world"] == WORLD and m1.global_step == STEPS
        torch.testing.assert_close(m1.table.reference_rows(), ref_rows, rtol=1e-5, atol=1e-7)
        # reference layout export/import round trip
        files = ckpt.export_reference_blocks(ckpt.latest_checkpoint(str(tmp_path / "log")), str(tmp_path / "ref"), 4)
        assert len(files) == 4
        m2 = FactorizationMachine(_cfg("local", "sum", 16), device="cpu")
        ckpt.import_reference_blocks(m2, str(tmp_path / "ref"), 4)
        assert torch.equal(m2.table.reference_rows(), _assemble(res))  # bit-exact round trip of the shards


@pytest.mark.parametrize("world,mode", [(4, "shard"), (8, "shard"), (4, "dp_dense"), (8, "dp_dense")])
def test_larger_worlds_equal_single_process(tmp_path, world, mode):
    """World 4 / 8 (the node sizes of the scaling runs): the sharded step with its N>1
    pipelining (depth-2 plan, early row exchange with dirty-row patches, split backward
    with per-owner halves) and the dense all-reduce mode equal one process on the
    concatenated batches; the W-shard checkpoint re-shards into one table."""
    res = _run_world(tmp_path, mode, "mean", 0, world)
    ref = _single("mean", world)
    ref_rows = ref.table.reference_rows()
    if mode == "shard":
        torch.testing.assert_close(_assemble(res), ref_rows, rtol=1e-5, atol=1e-7)
        m1 = FactorizationMachine(_cfg("local", "sum", 16), device="cpu")
        meta = ckpt.restore_checkpoint(m1, ckpt.latest_checkpoint(str(tmp_path / "log")))
        assert meta["shard_world"] == world
        torch.testing.assert_close(m1.table.reference_rows(), ref_rows, rtol=1e-5, atol=1e-7)
    else:
        for r in res:
            torch.testing.assert_close(r["rows"], ref_rows, rtol=1e-5, atol=1e-7)
        _check_dense_checkpoint(tmp_path, ref)
    for rank, r in enumerate(res):
        torch.testing.assert_close(r["pred"], ref.predict(_batch(99, rank)), rtol=1e-5, atol=1e-6)


def _check_dense_checkpoint(tmp_path, ref):
    """dp_dense keeps each row's optimizer state on its slice's owner only (sharded apply); the
    checkpoint all-gathers it first, so the restored table matches one process in rows AND state."""
    m1 = FactorizationMachine(_cfg("local", "sum", 16), device="cpu")
    ckpt.restore_checkpoint(m1, ckpt.latest_checkpoint(str(tmp_path / "log")))
    torch.testing.assert_close(m1.table.reference_rows(), ref.table.reference_rows(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(m1.table.s0v[:V, :KF], ref.table.s0v[:V, :KF], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(m1.table.s0w[:V], ref.table.s0w[:V], rtol=1e-5, atol=1e-7)
