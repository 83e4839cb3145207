"""Numerics of the native FM kernels (CPU and gfx950) against the fp64 PyTorch oracle.

The scorer fixture ports the semantic test vectors of the reference's
test/fm_scorer_op_test.py:9-78 (B=2, K=8, vocab 10 + zero padding row 0,
duplicate id 2 in example 0, random params U(0.01, 0.02), MSE-sum cost + reg,
gradient w.r.t. the whole params matrix).
"""

import pytest
import torch

from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K
from fast_tffm_amd.ops.fm_ops import fm_scorer

from oracle import fm_scores, ftrl_step, reference_train_step

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _params_ref(model) -> torch.Tensor:
    return model.table.reference_rows().double().cpu()


@pytest.mark.parametrize("device", DEVICES)
def test_scorer_fixture_matches_dense_reference(device):
    torch.manual_seed(7)
    factor_num, vocab = 8, 10
    feature_ids = [[1, 2, 3, 2, 4, 9], [3, 4, 7, 0, 0, 0]]
    feature_vals = [[9.0, 2.0, 3.6, 4.0, -2.2, -10.7], [4.0, -3.4, 2.0, 0, 0, 0]]
    labels = torch.tensor([1.0, -1.0], dtype=torch.float64)
    lf, lb = 1.2, 0.4
    params = torch.cat([torch.zeros(1, factor_num + 1), torch.rand(vocab, factor_num + 1) * 0.01 + 0.01]).double()
    flat_ids, flat_vals, poses = [], [], [0]
    for i in range(2):
        for fid, fv in zip(feature_ids[i], feature_vals[i]):
            if fid == 0:
                continue
            flat_ids.append(fid)
            flat_vals.append(fv)
        poses.append(len(flat_ids))

    # dense reference (gather + reduce_sum), as in the reference test
    p_ref = params.clone().requires_grad_(True)
    ids_t = torch.tensor(feature_ids)
    fv_t = torch.tensor(feature_vals, dtype=torch.float64)
    factors = p_ref[:, 1:][ids_t]
    biases = p_ref[:, 0][ids_t]
    fs = (factors * fv_t[..., None]).sum(1)
    ref_pred = 0.5 * (fs * fs).sum(1) - 0.5 * (fv_t[..., None] ** 2 * factors ** 2).sum((1, 2)) + (biases * fv_t).sum(1)
    ref_reg = 0.5 * (lf * (factors * factors).sum() + lb * (biases * biases).sum())
    ref_cost = ((labels - ref_pred) ** 2).sum() + ref_reg
    (ref_grad,) = torch.autograd.grad(ref_cost, p_ref)

    p = params.float().to(device).requires_grad_(True)
    pred, reg = fm_scorer(torch.tensor(flat_ids, device=device), p, torch.tensor(flat_vals, device=device),
                          torch.tensor(poses, device=device), lf, lb)
    cost = ((labels.float().to(device) - pred) ** 2).sum() + reg
    (grad,) = torch.autograd.grad(cost, p)
    torch.testing.assert_close(pred.double().cpu(), ref_pred.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(reg.double().cpu(), ref_reg.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(grad.double().cpu(), ref_grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("factor_num", [4, 10, 16, 64, 100, 128])
@pytest.mark.parametrize("loss", ["mse", "logistic"])
def test_forward_and_loss(device, factor_num, loss):
    V = 500
    b = random_batch(96, V, max_feats=70, seed=factor_num, device=device,
                     label_kind="binary" if loss == "logistic" else "real")
    cfg = FMConfig(vocabulary_size=V, factor_num=factor_num, loss_type=loss, init_value_range=0.3, seed=3)
    m = FactorizationMachine(cfg, device=device)
    fo = m.forward(b, loss=loss, want_reg=True)
    pref, rv, rw = fm_scores(_params_ref(m), b.offsets.cpu(), b.ids.cpu(), b.vals.cpu())
    torch.testing.assert_close(fo.pred.double().cpu(), pref, rtol=2e-5, atol=2e-5)
    y = b.labels.cpu().double()
    wt = b.weights.cpu().double()
    if loss == "mse":
        per = wt * (pref - y) ** 2
    else:
        per = wt * torch.nn.functional.binary_cross_entropy_with_logits(pref, y, reduction="none")
    assert abs(float(fo.loss_sum) - float(per.sum())) <= 1e-4 * max(1.0, abs(float(per.sum())))
    assert abs(float(fo.regv) - float(rv)) <= 1e-4 * max(1.0, float(rv))
    assert abs(float(fo.regw) - float(rw)) <= 1e-4 * max(1.0, float(rw))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("factor_num", [8, 64, 100])
@pytest.mark.parametrize("loss", ["mse", "logistic"])
def test_train_step_matches_reference_adagrad(device, factor_num, loss):
    V = 300
    b = random_batch(64, V, max_feats=20, seed=11 + factor_num, device=device,
                     label_kind="binary" if loss == "logistic" else "real")
    cfg = FMConfig(vocabulary_size=V, factor_num=factor_num, loss_type=loss, factor_lambda=0.3, bias_lambda=0.2,
                   batch_size=50, init_value_range=0.2, seed=5,
                   opt=K.OptConfig("adagrad", lr=0.05, initial_accumulator=0.1))
    m = FactorizationMachine(cfg, device=device)
    p0 = _params_ref(m)
    acc0 = torch.full_like(p0, 0.1)
    out = m.train_step(b)
    p1, _, loss_ref = reference_train_step(p0, acc0, b.to("cpu"), loss, 0.05,
                                           0.3, 0.2, 50)
    torch.testing.assert_close(_params_ref(m), p1, rtol=1e-4, atol=2e-6)
    assert abs(out.mean_loss() - loss_ref) < 1e-4 * max(1.0, abs(loss_ref))


@pytest.mark.parametrize("device", DEVICES)
def test_hot_ids_multi_chunk_segments(device):
    """Many occurrences of a few ids (> the backward chunk size): exercises the chunk/combine path."""
    V, B = 50, 400
    g = torch.Generator().manual_seed(0)
    sizes = torch.full((B,), 6, dtype=torch.int32)
    offsets = torch.zeros(B + 1, dtype=torch.int32)
    offsets[1:] = torch.cumsum(sizes, 0)
    ids = torch.randint(0, 3, (B * 6,), generator=g)  # 3 hot ids, ~800 occurrences each
    ids[::7] = torch.randint(0, V, ids[::7].shape, generator=g)
    from fast_tffm_amd.data.batch import Batch

    b = Batch(torch.randn(B, generator=g), offsets, ids, torch.rand(B * 6, generator=g), None).to(device)
    cfg = FMConfig(vocabulary_size=V, factor_num=16, loss_type="mse", init_value_range=0.1, seed=2,
                   opt=K.OptConfig("adagrad", lr=0.02), dedup_chunk=32)
    m = FactorizationMachine(cfg, device=device)
    p0 = _params_ref(m)
    m.train_step(b)
    p1, _, _ = reference_train_step(p0, torch.full_like(p0, 0.1), b.to("cpu"), "mse", 0.02, 0.0, 0.0, cfg.batch_size)
    torch.testing.assert_close(_params_ref(m), p1, rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("device", DEVICES)
def test_ftrl_step(device):
    V = 200
    b = random_batch(50, V, max_feats=12, seed=3, device=device)
    opt = K.OptConfig("ftrl", lr=0.1, l1=0.01, l2=0.02, beta=1.0, initial_accumulator=0.1)
    cfg = FMConfig(vocabulary_size=V, factor_num=8, loss_type="logistic", init_value_range=0.2, seed=9, opt=opt)
    m = FactorizationMachine(cfg, device=device)
    p0 = _params_ref(m).clone().requires_grad_(True)
    from oracle import fm_objective, touched_rows

    obj, _, _ = fm_objective(p0, b.to("cpu"), "logistic", 0, 0, cfg.batch_size)
    (gr,) = torch.autograd.grad(obj, p0)
    t = touched_rows(b, V)
    p1, _, _ = ftrl_step(p0.detach(), torch.full_like(gr, 0.1), torch.zeros_like(gr), gr, t, 0.1, 0.01, 0.02, 1.0)
    m.train_step(b)
    torch.testing.assert_close(_params_ref(m), p1, rtol=1e-4, atol=2e-6)


@pytest.mark.parametrize("device", DEVICES)
def test_dedup_matches_torch_unique(device):
    g = torch.Generator().manual_seed(1)
    keys = torch.randint(0, 1000, (5000,), generator=g, dtype=torch.int32).to(device)
    ex = torch.arange(5000, dtype=torch.int32, device=device)
    dd = K.dedup(keys, key_bits=10, ex_of_occ=ex, want_inv=True)
    U = dd.sync()
    ref_u, ref_inv, ref_cnt = torch.unique(keys.cpu(), return_inverse=True, return_counts=True)
    assert U == ref_u.numel()
    assert torch.equal(dd.uniq[:U].cpu(), ref_u.to(torch.int32))
    assert torch.equal(dd.inv[:5000].cpu(), ref_inv.to(torch.int32))
    seg = dd.seg_start[: U + 1].cpu()
    assert torch.equal(seg[1:] - seg[:-1], ref_cnt.to(torch.int32))
    # stable: within a segment occurrences stay in input order
    se = dd.sorted_ex[:5000].cpu()
    for u in range(0, U, 97):
        s = se[seg[u]:seg[u + 1]]
        assert torch.all(s[1:] > s[:-1])


@pytest.mark.parametrize("device", DEVICES)
def test_bf16_table_forward(device):
    V = 400
    b = random_batch(64, V, max_feats=30, seed=4, device=device)
    cfg = FMConfig(vocabulary_size=V, factor_num=64, dtype=torch.bfloat16, init_value_range=0.2, seed=1)
    m = FactorizationMachine(cfg, device=device)
    fo = m.forward(b)
    pref, _, _ = fm_scores(_params_ref(m), b.offsets.cpu(), b.ids.cpu(), b.vals.cpu())
    torch.testing.assert_close(fo.pred.double().cpu(), pref, rtol=1e-4, atol=1e-4)


def test_seg_index_sizing_and_lookup_contract():
    """Key-bucket segment index (hip/dedup.hip seg_index_kernel; the row-sharded forward's
    key -> segment lookup): sizing, and the build / lookup contract emulated in numpy -- every
    bucket written exactly once (no clear), keys found in [idx[b], idx[b + 1])."""
    import numpy as np

    shift, nb = K.seg_index_bits(5_111_808, 27)
    assert nb == 1 << 20 and shift == 7
    assert K.seg_index_bits(100, 16) == (11, 32)      # ~nnz / 4 buckets, a power of two
    assert K.seg_index_bits(10, 16) == (12, 16)       # at least 16
    assert K.seg_index_bits(1 << 30, 12) == (0, 4096)  # never more buckets than keys
    rng = np.random.default_rng(0)
    for key_bits, n in ((20, 40000), (27, 100000), (16, 3000)):
        keys = np.unique(rng.integers(0, (1 << key_bits) * 3 // 4, n))  # top of the range unused
        shift, nb = K.seg_index_bits(n, key_bits)
        U = len(keys)
        idx = np.full(nb + 1, -1, np.int64)
        writes = np.zeros(nb + 1, np.int64)
        for s in range(U):  # the kernel's per-segment loop
            lo = 0 if s == 0 else (keys[s - 1] >> shift) + 1
            hi = keys[s] >> shift
            idx[lo:hi + 1] = s
            writes[lo:hi + 1] += 1
        tail0 = (keys[-1] >> shift) + 1  # the grid-strided tail
        idx[tail0:] = U
        writes[tail0:] += 1
        assert bool((writes == 1).all())
        b = keys >> shift
        lo, hi = idx[b], idx[b + 1]
        seg = np.arange(U)
        assert bool(((seg >= lo) & (seg < hi)).all())


def test_fp8_row_scale_is_power_of_two():
    """quantize_fp8_rows (the kernels' store_row rule): s = the power of two with max|v| / s in
    (224, 448]; 1 for empty rows; the quantised row reproduces v within half an e4m3 step."""
    g = torch.Generator().manual_seed(3)
    v = torch.randn(257, 40, generator=g) * torch.logspace(-6, 3, 257).unsqueeze(1)
    v[5] = 0.0
    v[6, :] = 0.0
    v[6, 3] = 448.0 * 2.0 ** -10  # exactly a power of two times 448: m / s == 448
    q, s = K.quantize_fp8_rows(v)
    mant, _ = torch.frexp(s)
    assert bool((mant == 0.5).all()) and float(s[5]) == 1.0 and float(s[6]) == 2.0 ** -10
    top = (v.abs().amax(1) / s)[v.abs().amax(1) > 0]
    assert bool((top > 224.0).all() and (top <= 448.0).all())
    err = (q.float() * s[:, None] - v).abs()
    assert bool((err <= 16.0 * s[:, None]).all())
