"""The row-sharded GPU executor at world 2-4 on ONE GPU.

RCCL refuses two ranks on one device, so the ranks talk over gloo through a relay:
``torch.distributed`` collectives / P2P ops called by the exchange on GPU tensors are
staged through host memory.  Everything else is the real multi-rank GPU path --
dedup + owner counts, run-merge apply over 2 runs, the early row exchange with its
dirty scan / compaction / tagged patch gather / patch scatter between two ranks, the
split backward with several owners and its send/recv pieces, depth-2 lookahead -- and
must equal one process training on the concatenated batches (grad_reduce = mean);
fp32 / bf16 / fp8 tables (the latter two travel as uint8 wire rows)."""

import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

V, KF, B, STEPS = 6007, 64, 512, 5


def _free_port() -> int:
    from ports import free_port

    return free_port()


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


def _install_relay():
    import torch.distributed as tdist

    real_a2a, real_isend, real_irecv = tdist.all_to_all_single, tdist.isend, tdist.irecv

    def a2a(out, inp, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
        if not (out.is_cuda or inp.is_cuda):
            return real_a2a(out, inp, output_split_sizes, input_split_sizes, group=group, async_op=async_op)
        o = torch.empty(out.shape, dtype=out.dtype)
        real_a2a(o, inp.cpu(), output_split_sizes, input_split_sizes, group=group)
        out.copy_(o)
        return _Done() if async_op else None

    def batch_isend_irecv(ops):
        works, recvs = [], []
        for op in ops:
            if op.op in (tdist.isend, real_isend):
                works.append(real_isend(op.tensor.cpu(), op.peer, group=op.group))
            else:
                buf = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
                works.append(real_irecv(buf, op.peer, group=op.group))
                recvs.append((op.tensor, buf))
        for w in works:
            w.wait()
        for t, buf in recvs:
            t.copy_(buf)
        return [_Done()]

    tdist.all_to_all_single = a2a
    tdist.batch_isend_irecv = batch_isend_irecv


def _cfg(mode, bcfg, **kw):
    from fast_tffm_amd.models.fm import FMConfig
    from fast_tffm_amd.ops import kernels as K

    kw = dict(kw)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": K.FP8}[kw.pop("dtype", "fp32")]
    return FMConfig(vocabulary_size=V, factor_num=KF, loss_type="logistic", factor_lambda=0.01, bias_lambda=0.01,
                    batch_size=bcfg, init_value_range=0.05, seed=11, mode=mode, grad_reduce="mean", dtype=dt,
                    stochastic_rounding=False, opt=K.OptConfig("adagrad", lr=0.05), **kw)


def _batch(step, rank):
    from fast_tffm_amd.data.synthetic import CriteoSynth

    return CriteoSynth(V, seed=1000 * step + rank, device="cuda").batch(B)


def _worker(rank, world, port, out_dir, variant):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _install_relay()
    from fast_tffm_amd.models.fm import FactorizationMachine
    from fast_tffm_amd.parallel import dist as fmdist

    variant = dict(variant)
    os.environ.update(variant.pop("env", {}))
    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cuda:0")
    m = FactorizationMachine(_cfg("shard", B, **variant), device="cuda:0", dist=ctx)
    bs = [_batch(s, rank) for s in range(STEPS)]
    losses = []
    for s in range(STEPS):
        nb = bs[s + 1] if s + 1 < STEPS else None
        nb2 = bs[s + 2] if s + 2 < STEPS else None
        losses.append(m.train_step(bs[s], nb, nb2).mean_loss())
    torch.cuda.synchronize()
    ex = m._exchange
    torch.save({"gids": m.table.global_ids().cpu(), "rows": m.table.reference_rows().cpu(), "losses": losses,
                "early": ex.early_steps, "split": ex.overlap_grads}, os.path.join(out_dir, f"rank{rank}.pt"))
    fmdist.shutdown()


@pytest.mark.parametrize("world,variant", [
    (2, dict()), (2, dict(prefetch_rows="off")), (4, dict()), (3, dict(dtype="bf16")), (2, dict(dtype="fp8")),
    (3, dict(overlap_grads="off")), (2, dict(overlap_grads="off", env={"FM_SELF_ROWS": "0"})),
    (3, dict(dtype="bf16", env={"FM_SELF_ROWS": "0"}))])
def test_ranks_on_one_gpu_equal_one_process(tmp_path, world, variant):
    """Self rows (the default) at world 2-4: each rank reads its own rows from its table and
    updates the ones no other rank requested in place; FM_SELF_ROWS=0 exchanges them too."""
    from fast_tffm_amd.data.batch import Batch
    from fast_tffm_amd.models.fm import FactorizationMachine

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), variant), nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    if "prefetch_rows" not in variant:  # default at world > 1: early row exchange on
        assert all(r["early"] == STEPS - 1 for r in res)
    assert all(r["split"] == (variant.get("overlap_grads", "auto") != "off") for r in res)  # (split: default on)
    ref = FactorizationMachine(_cfg("local", B * world, dtype=variant.get("dtype", "fp32")), device="cuda")
    for s in range(STEPS):
        parts = [_batch(s, r) for r in range(world)]
        offs = torch.cat([parts[0].offsets] + [p.offsets[1:] + parts[0].nnz * i  # (every part: B x 39 features)
                                               for i, p in enumerate(parts[1:], 1)])
        ref.train_step(Batch(torch.cat([p.labels for p in parts]), offs, torch.cat([p.ids for p in parts]), None, None,
                             sum(p.nnz for p in parts)))
    torch.cuda.synchronize()
    want = ref.table.reference_rows().cpu()
    got = torch.zeros_like(want)
    for r in res:
        g = r["gids"]
        ok = g < V
        got[g[ok]] = r["rows"][ok]
    tol = dict(rtol=1e-5, atol=1e-6) if variant.get("dtype", "fp32") == "fp32" else dict(rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(got, want, **tol)
