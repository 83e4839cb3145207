"""Fused singleton update (fm_fwd.hip fwd_single_update): rows that occur once in a batch
get their optimizer step in the forward kernel, and the backward skips their one-occurrence
chunks.  The gradient is formed exactly as the chunk kernel forms it, so the table after a
run of lookahead steps must be bitwise identical to the unfused run (FM_FWD_SINGLE=0) for
every table dtype and optimizer; the fp32 path is also checked against the fp64 oracle."""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth, random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

from oracle import reference_train_step

pytestmark = pytest.mark.gpu


def _model(dtype, opt, k=64, V=200_000):
    cfg = FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=11,
                   opt=opt, batch_size=4096, factor_lambda=0.01, bias_lambda=0.01, dtype=dtype)
    return FactorizationMachine(cfg, device="cuda")


def _run(monkeypatch, fused, dtype, opt, k, batches):
    monkeypatch.setenv("FM_FWD_SINGLE", "1" if fused else "0")
    m = _model(dtype, opt, k)
    losses = []
    for i, b in enumerate(batches):
        nb = batches[i + 1] if i + 1 < len(batches) else None
        losses.append(m.train_step(b, nb).mean_loss())
    torch.cuda.synchronize()
    st = m.table.state
    out = {n: getattr(st, n).clone() for n in ("v", "w", "s0v", "s1v", "s0w", "s1w") if getattr(st, n) is not None}
    m.close()
    return losses, out


@pytest.mark.parametrize("dtype,opt,k", [
    (torch.float32, K.OptConfig("adagrad", lr=0.05), 64),
    (torch.bfloat16, K.OptConfig("adagrad", lr=0.05), 16),
    (torch.float8_e4m3fn, K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0), 128),
    (torch.float32, K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0), 32),
])
def test_fused_singletons_bitwise_equal_unfused(monkeypatch, dtype, opt, k):
    gen = CriteoSynth(200_000, seed=3, device="cuda")
    batches = [gen.batch(4096) for _ in range(4)]
    # the dedup flags must find singletons for the test to mean anything
    m = _model(dtype, opt, k)
    monkeypatch.setenv("FM_FWD_SINGLE", "1")
    rows, dd = m._plan_into(m._lslots[0], batches[0])
    torch.cuda.synchronize()
    assert dd.single_flag is not None
    ids = batches[0].ids.long()
    _, inv, cnt = torch.unique(ids, return_inverse=True, return_counts=True)
    want = (cnt[inv] == 1).to(torch.uint8)
    assert torch.equal(dd.single_flag[: ids.numel()], want)
    assert int(want.sum()) > 1000
    m.close()
    la, ta = _run(monkeypatch, False, dtype, opt, k, batches)
    lb, tb = _run(monkeypatch, True, dtype, opt, k, batches)
    for n in ta:
        x, y = ta[n], tb[n]
        ne = (x.view(torch.uint8) != y.view(torch.uint8))
        if bool(ne.any()):
            d = (x.float() - y.float()).abs()
            pytest.fail(f"{n}: {int(ne.sum())} bytes differ, max |diff| {float(d.max()):.3g}")
    assert la == lb


def test_fused_singletons_match_oracle(monkeypatch):
    """Valued, weighted features (x != 1: the occurrence-payload dedup) against the fp64 oracle."""
    monkeypatch.setenv("FM_FWD_SINGLE", "1")
    cfg = FMConfig(vocabulary_size=3000, factor_num=16, loss_type="logistic", init_value_range=0.05, seed=3,
                   opt=K.OptConfig("adagrad", lr=0.05), batch_size=512, factor_lambda=0.01, bias_lambda=0.01)
    m = FactorizationMachine(cfg, device="cuda")
    b = random_batch(512, 3000, max_feats=30, seed=4, device="cuda")
    rows, dd = m._plan_into(m._lslots[0], b)
    torch.cuda.synchronize()
    assert dd.single_flag is not None and int(dd.single_flag[: b.nnz].sum()) > 50
    p0 = m.table.reference_rows().double().cpu()
    m.train_step(b)
    p1, _, _ = reference_train_step(p0, torch.full_like(p0, 0.1), b.to("cpu"), "logistic", 0.05, 0.01, 0.01, 512)
    torch.testing.assert_close(m.table.reference_rows().double().cpu(), p1, rtol=2e-4, atol=5e-6)
    m.close()
