"""The wide fp8 chunk backward (hip/fm_bwd.hip, FM_FP8_WIDE: k=128 fp8 rows reduced with 8 values per
lane, 16-byte r1 / state accesses) against the 4-value kernel it replaces, built as the "fp8narrow"
variant: local training steps must leave every byte of the table -- fp8 rows, [w, scale, norm] rows,
bf16 optimizer state -- identical (same per-element arithmetic, stochastic-rounding columns and norm
butterfly: fm_common.h store_row_fp8x8).  Adagrad and FTRL, with and without feature values, batches
with single-occurrence rows (short block), mid-length chunks and hot rows (partials + combines).
"""

import os

import pytest
import torch

from fast_tffm_amd.data.batch import Batch
from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

V, B, STEPS = 60_000, 8192, 4


def _batches(with_vals: bool):
    gen = CriteoSynth(V, seed=13, device="cuda")
    out = []
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(STEPS):
        b = gen.batch(B)
        if with_vals:
            vals = torch.rand(b.nnz, generator=g, device="cuda") * 2.0
            b = Batch(b.labels, b.offsets, b.ids, vals, None, b.nnz, max_feats=b.max_feats)
        out.append(b)
    return out


def _train(opt: str, batches, dist=None, split="auto"):
    o = K.OptConfig("ftrl", lr=0.05, l1=0.01, l2=0.01, beta=1.0) if opt == "ftrl" else K.OptConfig("adagrad", lr=0.05)
    cfg = FMConfig(vocabulary_size=V, factor_num=128, loss_type="logistic", batch_size=B, init_value_range=0.05, seed=3,
                   opt=o, dtype=K.FP8, factor_lambda=0.001, bias_lambda=0.001, mode="shard" if dist else "local",
                   overlap_grads=split)
    m = FactorizationMachine(cfg, device="cuda", dist=dist)
    for i, b in enumerate(batches):
        m.train_step(b, *batches[i + 1: i + 3]) if dist else m.train_step(b)
    torch.cuda.synchronize()
    t = m.table  # (wx: [w, scale, |v|^2, pad] per fp8 row)
    out = [x.clone() for x in (t.v, t.wx, t.s0v, t.s0w, t.s1v, t.s1w) if x is not None]
    m.close()
    return out


@pytest.mark.parametrize("opt", ["adagrad", "ftrl"])
@pytest.mark.parametrize("with_vals", [False, True])
def test_wide_fp8_backward_is_bitwise_the_narrow_one(opt, with_vals, monkeypatch):
    from fast_tffm_amd.ops import native

    batches = _batches(with_vals)
    monkeypatch.delenv("FM_HIP_VARIANT", raising=False)
    n0 = native.hip().bwd_wide_launches()
    wide = _train(opt, batches)
    assert native.hip().bwd_wide_launches() - n0 == STEPS  # (the wide kernel ran every step)
    monkeypatch.setenv("FM_HIP_VARIANT", "fp8narrow")
    try:
        native.hip()
    except native.NativeExtensionError as e:
        pytest.skip(f"fp8narrow build variant not available: {e}")
    narrow = _train(opt, batches)
    assert native.hip().bwd_wide_launches() == 0
    assert len(wide) == len(narrow)
    names = ["v", "wx", "s0v", "s0w", "s1v", "s1w"][: len(wide)]
    bad = {}
    for n, a, b in zip(names, wide, narrow):
        assert a.dtype == b.dtype and a.shape == b.shape
        d = (a.view(torch.uint8) != b.view(torch.uint8))
        if bool(d.any()):
            fa, fb = a.float(), b.float()
            bad[n] = (int(d.sum()), float((fa - fb).abs().max()), float(fa.abs().max()))
    assert not bad, bad


@pytest.fixture(scope="module")
def rccl_ctx():
    from ports import free_port

    from fast_tffm_amd.parallel import dist as fmdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    ctx = fmdist.init_distributed(backend="nccl", rank=0, world=1, device="cuda:0", force_pg=True)
    yield ctx
    fmdist.shutdown()


@pytest.mark.parametrize("self_rows", ["1", "0"])
@pytest.mark.parametrize("split", ["on", "off"])
def test_wide_fp8_emit_backward_is_bitwise_the_narrow_one(rccl_ctx, self_rows, split, monkeypatch):
    """The row-sharded step's EMIT kernels (RCCL world 1 on the N > 1 compute path): own rows updated in
    place (self rows) or every row as a gradient row through the owner's apply, one pass or the split
    backward's two pieces."""
    from fast_tffm_amd.ops import native

    monkeypatch.setenv("FM_SHARD_W1_LOCAL", "0")
    monkeypatch.setenv("FM_SELF_ROWS", self_rows)
    batches = _batches(True)
    monkeypatch.delenv("FM_HIP_VARIANT", raising=False)
    n0 = native.hip().bwd_wide_launches()
    wide = _train("ftrl", batches, rccl_ctx, split)
    assert native.hip().bwd_wide_launches() > n0
    monkeypatch.setenv("FM_HIP_VARIANT", "fp8narrow")
    try:
        native.hip()
    except native.NativeExtensionError as e:
        pytest.skip(f"fp8narrow build variant not available: {e}")
    narrow = _train("ftrl", batches, rccl_ctx, split)
    for n, a, b in zip(["v", "wx", "s0v", "s0w", "s1v", "s1w"], wide, narrow):
        assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), n
