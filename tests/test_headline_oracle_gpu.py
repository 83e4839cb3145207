"""One training step at the headline bench's shape against an fp64 oracle computed on the GPU.

Elsewhere the oracle tests run at B <= 2048 and vocabularies <= 20k (tests/test_kernels.py,
tests/test_step_gpu.py).  The bench's shape exercises what those cannot: ~5.1M occurrences,
hot rows of Criteo's low-cardinality fields with ~40k occurrences each (many chunks per row:
the lane-group combine and the workgroup "big row" reduction), 32-bit row addressing over a
10M-row table and the 131072-example r1 cache.  The oracle is reference FmScorer + FmGrad +
SparseApplyAdagrad / FTRL semantics (tests/oracle.py; reference cc/fm_scorer_op.h:8-140,
cc/fm_grad_op.h:59-163, tffm/fm_model.py:311-348) evaluated in fp64 with autograd on the
touched rows only, gathered per occurrence on the GPU.

(a) k=64 fp32 table + Adagrad: every touched row and its accumulator within the fp32 summation
    bound of the hottest rows' ~40k-term gradient sums.
(b) k=128 fp8 table + FTRL (BASELINE config 5): the fp32 linear weights tightly, the fp8 factors
    within the requantisation bound (one e4m3 step at the row's stored power-of-two scale, plus
    the bf16 r1 cache's 2^-9 relative error carried into the FTRL closed form).

Both on the local step and on the row-sharded step's N > 1 compute path run at world 1 ("emit":
RCCL world 1, FM_SHARD_W1_LOCAL=0 -- the sharded forward with self rows and the segment lookup, the
EMIT-specialised chunk kernels with in-place self-row updates, the plan chain with the fused
sharded-key sort).
"""

import os


import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

V, B = 10_000_000, 131072
LAMBDA_F, LAMBDA_B = 0.01, 0.01


@pytest.fixture(scope="module")
def rccl_ctx():
    from ports import free_port

    from fast_tffm_amd.parallel import dist as fmdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    ctx = fmdist.init_distributed(backend="nccl", rank=0, world=1, device="cuda:0", force_pg=True)
    yield ctx
    fmdist.shutdown()


def _model(cfg, path, request, monkeypatch):
    """The local step, or ("emit") the row-sharded N > 1 compute path at RCCL world 1."""
    if path == "local":
        return FactorizationMachine(cfg, device="cuda")
    monkeypatch.setenv("FM_SHARD_W1_LOCAL", "0")
    ctx = request.getfixturevalue("rccl_ctx")
    cfg.mode = "shard"
    m = FactorizationMachine(cfg, device="cuda", dist=ctx)
    assert not m._exchange.local_w1 and m._exchange.self_rows
    return m


@pytest.fixture
def production(monkeypatch):
    """FM_DEBUG_CHECKS off, as in bench.py (no host reads inside the kernel wrappers)."""
    was = K.debug_checks()
    K.set_debug_checks(False)
    monkeypatch.setenv("FM_DEBUG_CHECKS", "0")
    yield
    K.set_debug_checks(was)


def _objective_grad(P: torch.Tensor, loc: torch.Tensor, b, K_: int):
    """fp64 gradient of loss + reg / B_cfg w.r.t. the touched rows P [U, K+1] (col 0 = w), the
    occurrences indexing P through ``loc``; returns (grad [U, K+1], mean loss)."""
    P = P.detach().clone().requires_grad_(True)
    ex = torch.repeat_interleave(torch.arange(b.B, device=P.device),
                                 (b.offsets[1:] - b.offsets[:-1]).long(), output_size=b.nnz)
    rows = P[loc]
    w, v = rows[:, 0], rows[:, 1:]
    lin = torch.zeros(b.B, dtype=P.dtype, device=P.device).index_add(0, ex, w)
    s1 = torch.zeros((b.B, K_), dtype=P.dtype, device=P.device).index_add(0, ex, v)
    s2 = torch.zeros((b.B, K_), dtype=P.dtype, device=P.device).index_add(0, ex, v * v)
    pred = lin + 0.5 * (s1 * s1 - s2).sum(1)
    y = b.labels.to(P.dtype)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(pred, y, reduction="mean")
    reg = 0.5 * LAMBDA_F * (v * v).sum() + 0.5 * LAMBDA_B * (w * w).sum()
    (g,) = torch.autograd.grad(loss + reg / b.B, P)
    return g, float(loss)


def _touched(b):
    ids = b.ids.long()
    uniq, loc = torch.unique(ids, return_inverse=True)
    return uniq, loc


@pytest.mark.parametrize("path", ["local", "emit"])
def test_headline_step_k64_fp32_adagrad_matches_fp64_oracle(production, path, request, monkeypatch):
    K_ = 64
    lr, acc0 = 0.01, 0.1
    cfg = FMConfig(vocabulary_size=V, factor_num=K_, loss_type="logistic", batch_size=B, init_value_range=0.01,
                   seed=42, factor_lambda=LAMBDA_F, bias_lambda=LAMBDA_B, mode="local",
                   opt=K.OptConfig("adagrad", lr=lr, initial_accumulator=acc0))
    m = _model(cfg, path, request, monkeypatch)
    gen = CriteoSynth(V, seed=1000, device="cuda")
    b, nb = gen.batch(B), gen.batch(B)
    uniq, loc = _touched(b)
    # the hot rows this test is about: Criteo's 3- / 4-value fields give rows with tens of thousands
    # of occurrences (many chunks: combine + big-row kernels)
    assert int(torch.bincount(loc).max()) > 20000
    P0 = m.table.reference_rows(uniq).double()
    out = m.train_step(b, nb)          # the bench's lookahead step (dedup on the side stream)
    torch.cuda.synchronize()
    g, loss = _objective_grad(P0, loc, b, K_)
    acc1 = acc0 + g * g
    P1 = P0 - lr * g / acc1.sqrt()
    got = m.table.reference_rows(uniq).double()
    got_acc = torch.cat([m.table.s0w[uniq].unsqueeze(1), m.table.s0v[uniq, :K_]], 1).double()
    assert abs(out.mean_loss() - loss) <= 1e-5 * abs(loss)
    # fp32 sums of up to ~40k terms (chunked in fixed order): the gradient's relative error stays
    # ~1e-5; Adagrad's first step moves a parameter by lr * g / sqrt(0.1 + g^2) <= lr
    torch.testing.assert_close(got_acc, acc1, rtol=2e-5, atol=1e-9)
    torch.testing.assert_close(got, P1, rtol=2e-5, atol=2e-7)
    # untouched rows stay put (a sample of them)
    rest = torch.randint(0, V, (100000,), device="cuda")
    rest = rest[~torch.isin(rest, uniq)]
    cfg.mode = "local"
    fresh = FactorizationMachine(cfg, device="cuda")
    assert torch.equal(m.table.reference_rows(rest), fresh.table.reference_rows(rest))
    m.close()
    fresh.close()


def _ftrl(p, n, z, g, alpha, l1, l2, beta):
    n_new = n + g * g
    sigma = (n_new.sqrt() - n.sqrt()) / alpha
    z = z + g - sigma * p
    quad = (beta + n_new.sqrt()) / alpha + 2 * l2
    p = torch.where(z.abs() > l1, (torch.sign(z) * l1 - z) / quad, torch.zeros_like(z))
    return p, n_new, z


@pytest.mark.parametrize("path", ["local", "emit"])
def test_headline_step_k128_fp8_ftrl_matches_oracle(production, path, request, monkeypatch):
    K_ = 128
    o = K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0, initial_accumulator=0.1)
    cfg = FMConfig(vocabulary_size=V, factor_num=K_, loss_type="logistic", batch_size=B, init_value_range=0.01,
                   seed=42, factor_lambda=LAMBDA_F, bias_lambda=LAMBDA_B, mode="local", dtype=K.FP8, opt=o)
    m = _model(cfg, path, request, monkeypatch)
    gen = CriteoSynth(V, seed=1001, device="cuda")
    b, nb = gen.batch(B), gen.batch(B)
    uniq, loc = _touched(b)
    t = m.table
    P0 = t.reference_rows(uniq).double()
    n0 = torch.cat([t.s0w[uniq].unsqueeze(1), t.s0v[uniq, :K_].float()], 1).double()
    z0 = torch.cat([t.s1w[uniq].unsqueeze(1), t.s1v[uniq, :K_].float()], 1).double()
    m.train_step(b, nb)
    torch.cuda.synchronize()
    g, _ = _objective_grad(P0, loc, b, K_)
    P1, _, _ = _ftrl(P0, n0, z0, g, o.lr, o.l1, o.l2, o.beta)
    got = t.reference_rows(uniq).double()
    # linear weights are fp32 (their gradient uses no r1): close to the oracle
    torch.testing.assert_close(got[:, 0], P1[:, 0], rtol=1e-4, atol=1e-7)
    # factors: stochastically rounded e4m3 at the row's stored power-of-two scale -- less than one
    # step of the value's binade (|v| / 8 for normals, scale * 2^-9 for subnormals) -- plus the bf16
    # r1 cache (2^-9 relative, carried through the FTRL closed form)
    ref = P1[:, 1:]
    scale = t.scale[uniq].double()[:, None]
    step = torch.maximum(ref.abs() / 8, scale * 2.0 ** -9)
    err = (got[:, 1:] - ref).abs()
    bound = step + 0.01 * ref.abs() + 1e-8
    bad = err > bound
    assert not bool(bad.any()), (int(bad.sum()), float((err - bound)[bad].max()))
    # and on average well inside it (stochastic rounding is unbiased)
    assert float((got[:, 1:] - ref).mean().abs()) < 1e-5
    m.close()
