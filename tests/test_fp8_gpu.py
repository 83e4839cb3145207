"""fp8 factor table (BASELINE config 5): OCP e4m3 rows with one fp32 scale per
row, dequantised in the kernels, re-quantised on every update.

Numerics are checked against the fp64 oracle run on the DEQUANTISED table, so
the only allowed error is the final re-quantisation (half an fp8 step of the
row's scale); the forward must match the oracle to fp32 rounding."""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth, random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

from oracle import fm_scores, reference_train_step

pytestmark = pytest.mark.gpu
FP8 = torch.float8_e4m3fn


def _model(V, k, dtype, opt=None, **kw):
    cfg = FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=5,
                   opt=opt or K.OptConfig("adagrad", lr=0.05), batch_size=512, factor_lambda=0.01,
                   bias_lambda=0.01, dtype=dtype, **kw)
    return FactorizationMachine(cfg, device="cuda")


def test_fp8_init_matches_torch_quantisation():
    """The init kernel's quantisation (v_cvt_pk_fp8_f32, RNE) == torch's float8_e4m3fn cast of the fp32 init."""
    m8, m32 = _model(4000, 128, FP8), _model(4000, 128, torch.float32)
    q, s = K.quantize_fp8_rows(m32.table.v.float())
    torch.testing.assert_close(m8.table.scale, s, rtol=1e-6, atol=0)
    same = (m8.table.v.view(torch.uint8) == q.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same  # (a scale 1-ulp apart may flip a tie)
    torch.testing.assert_close(m8.table.w, m32.table.w)
    # dequantised values stay within half an e4m3 step of the fp32 init
    err = (m8.table.dense_v() - m32.table.v).abs()
    assert bool((err <= 16.0 * m8.table.scale[:, None] + 1e-12).all())


@pytest.mark.parametrize("k", [16, 128])
def test_fp8_forward_matches_oracle_on_dequantised_table(k):
    m = _model(3000, k, FP8)
    b = random_batch(256, 3000, max_feats=40, seed=3, device="cuda")
    p = m.table.reference_rows().double().cpu()
    pred = m.predict(b).double().cpu()
    ref, _, _ = fm_scores(p, b.offsets.cpu(), b.ids.cpu(), b.vals.cpu())
    torch.testing.assert_close(pred, ref, rtol=1e-5, atol=1e-6)


def test_fp8_adagrad_step_within_requantisation_error():
    V = 5000
    gen = CriteoSynth(V, device="cuda", seed=9)
    b = gen.batch(2048)
    m = _model(V, 64, FP8, stochastic_rounding=False)  # the bound below is round-to-nearest's
    p0 = m.table.reference_rows().double().cpu()
    m.train_step(b)
    p1, _, _ = reference_train_step(p0, torch.full_like(p0, 0.1), b.to("cpu"), "logistic", 0.05, 0.01, 0.01, 512)
    got = m.table.reference_rows().double().cpu()
    torch.testing.assert_close(got[:, 0], p1[:, 0], rtol=2e-4, atol=5e-6)  # w stays fp32
    scale = m.table.scale.double().cpu()[:, None]
    err = (got[:, 1:] - p1[:, 1:]).abs()
    assert bool((err <= 16.0 * scale * 1.01 + 1e-7).all()), float((err / scale).max())


def test_fp8_ftrl_trains_like_bf16():
    """k=128 fp8 + FTRL (config 5): the loss trajectory follows the bf16 table's."""
    V = 20000
    gen = CriteoSynth(V, device="cuda", seed=10)
    batches = [gen.batch(4096) for _ in range(8)]
    opt = K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0, initial_accumulator=0.1)
    m8, m16 = _model(V, 128, FP8, opt), _model(V, 128, torch.bfloat16, opt)
    l8 = [m8.train_step(bt).mean_loss() for bt in batches]
    l16 = [m16.train_step(bt).mean_loss() for bt in batches]
    assert l8[-1] < l8[0]
    for a, c in zip(l8, l16):
        assert abs(a - c) < 0.02 * max(1.0, abs(c)), (l8, l16)


def test_fp8_checkpoint_round_trip_is_exact(tmp_path):
    from fast_tffm_amd.utils import checkpoint as ckpt

    m = _model(3000, 32, FP8)
    m.train_step(random_batch(128, 3000, seed=1, device="cuda"))
    path = ckpt.save_checkpoint(m, str(tmp_path), 1)
    m2 = _model(3000, 32, FP8)
    m2.table.v.zero_()
    ckpt.restore_checkpoint(m2, path)
    assert torch.equal(m2.table.v.view(torch.uint8), m.table.v.view(torch.uint8))
    assert torch.equal(m2.table.wx, m.table.wx)
    # and into an fp32 table: the dequantised values
    m3 = _model(3000, 32, torch.float32)
    ckpt.restore_checkpoint(m3, path)
    torch.testing.assert_close(m3.table.reference_rows(), m.table.reference_rows())


def test_fp8_row_norms_track_stored_rows():
    """Every fp8 writer keeps [w, scale, |v|^2]: power-of-two scales, and the norm column equals the
    stored rows' squared norm -- bitwise the refresh kernel's (the same reduction)."""
    V = 6000
    gen = CriteoSynth(V, device="cuda", seed=12)
    opt = K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0, initial_accumulator=0.1)
    m = _model(V, 128, FP8, opt)
    t = m.table
    init_norm = t.norm2.clone()
    for _ in range(3):
        m.train_step(gen.batch(2048))
    torch.cuda.synchronize()
    mant, _ = torch.frexp(t.scale)
    assert bool((mant == 0.5).all())
    ref = (t.dense_v().double() ** 2).sum(1)
    torch.testing.assert_close(t.norm2.double(), ref, rtol=1e-6, atol=1e-12)
    assert not torch.equal(t.norm2, init_norm)  # (updated rows changed theirs)
    kept = t.norm2.clone()
    t.refresh_norms()
    assert torch.equal(t.norm2, kept)


def test_fp8_rows_with_free_scales_are_requantised():
    """Rows restored with scales that are not powers of two (a checkpoint of an older build; the
    restore calls Table.adopt_fp8_rows) are re-quantised from their dequantised values: the
    forward's scaled conversion reads only a scale's exponent."""
    m = _model(3000, 32, FP8)
    t = m.table
    vals = t.dense_v()[:, : t.K].clone()
    mx = vals.abs().amax(1)
    s = torch.where(mx > 0, mx / K.FP8_MAX, torch.ones_like(mx))  # the older rule: max / 448
    q = torch.zeros(t.v.shape, dtype=torch.float32, device=t.v.device)
    q[:, : t.K] = vals / s[:, None]
    t.v.copy_(q.clamp(-K.FP8_MAX, K.FP8_MAX).to(FP8))
    t.scale.copy_(s)
    before = t.dense_v().clone()
    t.adopt_fp8_rows()
    mant, _ = torch.frexp(t.scale)
    assert bool((mant == 0.5).all())
    err = (t.dense_v() - before).abs()
    assert bool((err <= 16.0 * t.scale[:, None] + 1e-12).all())
    torch.testing.assert_close(t.norm2.double(), (t.dense_v().double() ** 2).sum(1), rtol=1e-6, atol=1e-12)
