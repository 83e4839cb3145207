"""Hot rows of the local step (hip/hot.hip + the fp32-MFMA dense-row GEMM, fm_bwd.hip).

* the filter keeps exactly the non-hot (key, packed code) pairs, in CSR order;
* a training run with hot rows (FM_HOT_ROWS=1, the default) matches the same run without them
  (FM_HOT_ROWS=0: every row through the sort-based dedup and the chunk backward) to fp32
  summation-order error, for Adagrad and FTRL, fp32 and bf16 tables (fp8: the losses);
* it is deterministic: two runs give bitwise-identical tables.
"""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _production_checks():
    K.set_debug_checks(False)
    yield
    K.set_debug_checks(True)


def test_hot_filter_keeps_non_hot_pairs_in_order():
    gen = CriteoSynth(1_000_000, seed=3, device=DEV)
    b = gen.batch(3000)
    ids = b.ids.to(torch.int32)
    u, c = torch.unique(ids, return_counts=True)
    hot_keys = u[torch.argsort(c, descending=True)[:200]]
    hot = K.HotRows.empty(DEV)
    hot.set(hot_keys)
    sb = 6
    nnz = ids.numel()
    keys = torch.full((nnz,), -1, dtype=torch.int32, device=DEV)
    codes = torch.full((nnz,), -1, dtype=torch.int32, device=DEV)
    gcnt = torch.zeros((b.B + 63) // 64, dtype=torch.int32, device=DEV)
    n_out = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.hot_filter(b.offsets, ids, hot, slot_bits=sb, gcnt=gcnt, keys_out=keys, codes_out=codes, n_out=n_out)
    torch.cuda.synchronize()
    keep = ~torch.isin(ids, hot_keys.to(torch.int32))
    sizes = (b.offsets[1:] - b.offsets[:-1]).long()
    ex = torch.repeat_interleave(torch.arange(b.B, device=DEV), sizes)
    slot = torch.arange(nnz, device=DEV) - b.offsets[:-1].long()[ex]
    ref_codes = ((ex << sb) | slot).to(torch.int32)
    n = int(n_out.item())
    assert n == int(keep.sum())
    assert torch.equal(keys[:n], ids[keep]) and torch.equal(codes[:n], ref_codes[keep])


def _run(monkeypatch, hot: str, dtype, opt, steps=12):
    monkeypatch.setenv("FM_HOT_ROWS", hot)
    cfg = FMConfig(vocabulary_size=2_000_000, factor_num=64, loss_type="logistic", batch_size=8192,
                   init_value_range=0.01, seed=7, dtype=dtype, opt=opt, mode="local")
    m = FactorizationMachine(cfg, device=DEV)
    gen = CriteoSynth(cfg.vocabulary_size, seed=11, device=DEV)
    pool = [gen.batch(8192) for _ in range(4)]
    losses = []
    for i in range(steps):
        out = m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])
        losses.append(out.mean_loss())
    torch.cuda.synchronize()
    used = m._hot is not None and m._hot.n_host > 0
    t = m.table
    state = [x.detach().float().clone() for x in (t.v, t.w, t.s0v, t.s0w) + ((t.s1v, t.s1w) if t.s1v is not None
                                                                            else ())]
    m.close()
    return losses, state, used


@pytest.mark.parametrize("dtype,opt", [(torch.float32, K.OptConfig("adagrad", lr=0.05)),
                                       (torch.bfloat16, K.OptConfig("adagrad", lr=0.05)),
                                       (torch.float32, K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001)),
                                       (K.FP8, K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001))],
                         ids=["fp32_adagrad", "bf16_adagrad", "fp32_ftrl", "fp8_ftrl"])
def test_hot_rows_match_the_plain_step(monkeypatch, dtype, opt):
    l0, s0, used0 = _run(monkeypatch, "0", dtype, opt)
    l1, s1, used1 = _run(monkeypatch, "1", dtype, opt)
    assert not used0 and used1
    ltol = 2e-3 if dtype == K.FP8 else 1e-4
    for a, b in zip(l0, l1):
        assert abs(a - b) <= ltol * abs(a), (l0, l1)
    if dtype == K.FP8:  # (stochastic rounding to 3 mantissa bits: one flip is a whole step; the losses say it)
        return
    tol = 1e-5 if dtype == torch.float32 else 2e-2  # (bf16: a 1-ulp rounding flip on a row is 2^-8)
    for a, b in zip(s0, s1):
        assert torch.allclose(a, b, rtol=tol, atol=tol * 1e-2), float((a - b).abs().max())


def test_hot_rows_are_deterministic(monkeypatch):
    opt = K.OptConfig("adagrad", lr=0.05)
    _, s0, used = _run(monkeypatch, "1", torch.float32, opt, steps=8)
    _, s1, _ = _run(monkeypatch, "1", torch.float32, opt, steps=8)
    assert used
    for a, b in zip(s0, s1):
        assert torch.equal(a, b)
