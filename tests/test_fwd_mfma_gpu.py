"""fp8 k=128 forward on the matrix cores (hip/fm_fwd_mfma.hip) against the VALU kernel and the fp64
oracle (reference FmScorer, cc/fm_scorer_op.h:101-140, on the dequantised table).

The MFMA kernel multiplies the rows' stored e4m3 bytes by a block-diagonal e5m2 matrix of the rows'
power-of-two scales, offset per 16-example tile by the tile's largest scale; these tests give the rows
scales spread over 2^-14 .. 2^3 (and some all-zero rows), ragged examples including empty ones, a
batch that is not a multiple of the tile, and a full 16 x 48-row tile.

The matrix cores' fp8 products are not accumulated exactly in fp32: the error grows with the spread of
the summed terms' magnitudes (measured with tools/probe/mfma_fwd_err.py: scores within 3.7e-7 of the
terms' magnitude sum at similar row scales, 3e-6 at a 2^4 spread, 2.2e-5 at 2^17; the VALU kernel:
<1e-7).  The bounds below are 1e-4 of that magnitude -- far below the e4m3 rows' own quantisation
step (2^-4 of a value), which is what an fp8 table trades for its bandwidth.
"""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth, random_batch
from fast_tffm_amd.models.table import FMTable
from fast_tffm_amd.ops import kernels as K

from oracle import fm_scores

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def mfma_variant(monkeypatch):
    """The matrix-core forward lives in the "mfma" build variant (python -m fast_tffm_amd.build_native
    --variant mfma), not in the default module; skipped where that variant is not built."""
    from fast_tffm_amd.ops import native

    monkeypatch.setenv("FM_HIP_VARIANT", "mfma")
    try:
        native.hip()
    except native.NativeExtensionError as e:
        pytest.skip(f"mfma build variant not available: {e}")


def _table(V: int, seed: int) -> FMTable:
    t = FMTable(V, 128, dtype=K.FP8, device="cuda", seed=seed, init_range=0.05)
    g = torch.Generator(device="cuda").manual_seed(seed)
    mag = torch.exp2(torch.randint(-14, 4, (V, 1), generator=g, device="cuda").float())
    vals = torch.randn((V, 128), generator=g, device="cuda") * mag
    vals[torch.rand(V, generator=g, device="cuda") < 0.05] = 0.0   # all-zero rows
    t.set_v(None, vals)
    t.w.copy_(torch.randn(V, generator=g, device="cuda") * 0.1)
    return t


def _fwd(t: FMTable, b, mfma: bool):
    was = K.set_fwd_mfma(mfma)
    try:
        out = K.fm_forward(b.offsets, b.ids.to(torch.int32), None, t.v, t.w, t.Kp, labels=b.labels, weights=b.weights,
                           loss="logistic", grad_scale=0.5, want_reg=True, max_feats=b.max_feats)
        torch.cuda.synchronize()
    finally:
        K.set_fwd_mfma(was)
    return out


def _magnitudes(t: FMTable, b):
    """fp64 per-example scale of the score's terms (sum |w| + 1/2 (sum_k (sum |v_k|)^2 + sum v^2)) and
    per-column sum |v_k|: the error bounds are relative to these."""
    p = t.reference_rows().double()
    ex = torch.repeat_interleave(torch.arange(b.B, device="cuda"), (b.offsets[1:] - b.offsets[:-1]).long(),
                                 output_size=b.ids.numel())
    rows = p[b.ids.long()].abs()
    lin = torch.zeros(b.B, dtype=p.dtype, device="cuda").index_add(0, ex, rows[:, 0])
    col = torch.zeros((b.B, t.K), dtype=p.dtype, device="cuda").index_add(0, ex, rows[:, 1:])
    sq = torch.zeros(b.B, dtype=p.dtype, device="cuda").index_add(0, ex, (rows[:, 1:] ** 2).sum(1))
    return lin + 0.5 * ((col ** 2).sum(1) + sq), col


def _compare(t: FMTable, b):
    a, m = _fwd(t, b, False), _fwd(t, b, True)
    mag, col = _magnitudes(t, b)
    bnd = 1e-4 * mag + 1e-6
    assert bool(((m.pred.double() - a.pred.double()).abs() <= bnd).all())
    p = t.reference_rows().double().cpu()
    ref, _, _ = fm_scores(p, b.offsets.cpu(), b.ids.cpu(), None)
    assert bool(((m.pred.double().cpu() - ref).abs() <= bnd.cpu()).all())
    # dpred = grad_scale * wt * (sigmoid(pred) - y): sigmoid' <= 1/4
    wt = b.weights.double() if b.weights is not None else torch.ones(b.B, dtype=torch.float64, device="cuda")
    assert bool(((m.dpred.double() - a.dpred.double()).abs() <= 0.125 * wt * bnd + 1e-7).all())
    assert abs(float(m.loss_sum) - float(a.loss_sum)) <= float((wt * bnd).sum()) + 1e-5 * abs(float(a.loss_sum))
    torch.testing.assert_close(m.regv, a.regv, rtol=1e-5, atol=0)
    torch.testing.assert_close(m.regw, a.regw, rtol=1e-5, atol=0)
    # r1 (bf16): one bf16 step of the value plus the matrix cores' accumulation error
    d = (m.r1.double() - a.r1.double()).abs()
    assert bool((d <= 2.0 ** -6 * a.r1.double().abs() + 5e-4 * col + 1e-30).all())
    return m


@pytest.mark.parametrize("B,max_feats", [(1000, 40), (333, 48), (16, 1)])
def test_mfma_forward_matches_valu_and_oracle(B, max_feats):
    t = _table(6000, seed=B)
    b = random_batch(B, 6000, max_feats=max_feats, min_feats=0, seed=B, device="cuda", with_vals=False)
    assert b.vals is None
    _compare(t, b)


def test_mfma_forward_full_tile_of_hot_rows():
    """16 examples x 48 features (the kernel's 768-row tile) drawn from 50 rows: many repeats per tile."""
    t = _table(50, seed=7)
    b = random_batch(64, 50, max_feats=48, min_feats=48, seed=7, device="cuda", with_vals=False)
    _compare(t, b)


def test_mfma_forward_on_criteo_shape():
    t = _table(100_000, seed=3)
    b = CriteoSynth(100_000, seed=3, device="cuda").batch(4096)
    _compare(t, b)


def test_mfma_forward_understated_max_feats_is_loud():
    t = _table(1000, seed=4)
    b = random_batch(64, 1000, max_feats=60, min_feats=60, seed=4, device="cuda", with_vals=False)
    b.max_feats = 40   # 16 x 60 rows > the 768-row tile: NaN scores, no LDS overrun
    was_dbg = K.debug_checks()
    K.set_debug_checks(False)
    try:
        out = _fwd(t, b, True)
    finally:
        K.set_debug_checks(was_dbg)
    assert bool(torch.isnan(out.pred).all())
