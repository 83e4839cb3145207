"""Step-level GPU properties: hipGraph replay == eager step, bitwise determinism, Criteo-shaped batches."""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth, random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

from oracle import reference_train_step

pytestmark = pytest.mark.gpu


def _model(V=20000, k=64, **kw):
    cfg = FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=3,
                   opt=K.OptConfig("adagrad", lr=0.05), batch_size=512, factor_lambda=0.01, bias_lambda=0.01, **kw)
    return FactorizationMachine(cfg, device="cuda")


def _state(m):
    t = m.table
    return [x.clone() for x in (t.v, t.w, t.s0v, t.s0w)]


def test_graph_replay_matches_eager_bitwise():
    gen = CriteoSynth(20000, device="cuda", seed=5)
    batches = [gen.batch(512) for _ in range(3)]
    a, b = _model(), _model()
    for bt in batches:
        a.train_step(bt)
    b.capture_graph(batches[0])
    losses = [b.train_step(bt).mean_loss() for bt in batches]
    torch.cuda.synchronize()
    for x, y in zip(_state(a), _state(b)):
        assert torch.equal(x, y)
    assert all(l == l for l in losses)


def test_step_is_deterministic():
    gen = CriteoSynth(20000, device="cuda", seed=6)
    batches = [gen.batch(1024) for _ in range(2)]
    runs = []
    for _ in range(2):
        m = _model()
        for bt in batches:
            m.train_step(bt)
        torch.cuda.synchronize()
        runs.append(_state(m))
    for x, y in zip(*runs):
        assert torch.equal(x, y)


def test_criteo_shaped_step_matches_oracle():
    """Hot ids (thousands of occurrences: the workgroup combine path) against the fp64 oracle."""
    V = 5000
    gen = CriteoSynth(V, device="cuda", seed=7)
    b = gen.batch(2048)
    m = _model(V=V, k=16)
    p0 = m.table.reference_rows().double().cpu()
    m.train_step(b)
    p1, _, _ = reference_train_step(p0, torch.full_like(p0, 0.1), b.to("cpu"), "logistic", 0.05, 0.01, 0.01, 512)
    torch.testing.assert_close(m.table.reference_rows().double().cpu(), p1, rtol=2e-4, atol=5e-6)


def test_bf16_table_step_close_to_fp32():
    b = random_batch(256, 3000, max_feats=40, seed=2, device="cuda")
    m32, m16 = _model(V=3000, k=64), _model(V=3000, k=64, dtype=torch.bfloat16)
    m32.train_step(b)
    m16.train_step(b)
    torch.testing.assert_close(m16.table.reference_rows(), m32.table.reference_rows(), rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("k,dtype", [(16, torch.float32), (64, torch.float32), (100, torch.float32),
                                     (64, torch.bfloat16), (128, torch.bfloat16)])
def test_lookahead_step_matches_oracle(k, dtype):
    """The lookahead step (dedup of the batch on the side stream ahead of its forward) against the
    fp64 oracle on a Criteo-shaped batch, k = 16..128, fp32 / bf16 tables."""
    V = 5000
    gen = CriteoSynth(V, device="cuda", seed=13)
    b, b2 = gen.batch(2048), gen.batch(2048)
    m = _model(V=V, k=k, dtype=dtype)
    p0 = m.table.reference_rows().double().cpu()
    m.train_step(b, b2)
    torch.cuda.synchronize()
    p1, _, _ = reference_train_step(p0, torch.full_like(p0, 0.1), b.to("cpu"), "logistic", 0.05, 0.01, 0.01, 512)
    got = m.table.reference_rows().double().cpu()
    if dtype == torch.float32:
        torch.testing.assert_close(got, p1, rtol=2e-4, atol=5e-6)
    else:
        torch.testing.assert_close(got, p1, rtol=2e-2, atol=2e-3)


def test_local_lookahead_matches_plain_steps_bitwise(monkeypatch):
    """Eager lookahead (next batch's dedup on the side stream during this step) == plain steps."""
    gen = CriteoSynth(20000, device="cuda", seed=15)
    batches = [gen.batch(1024) for _ in range(4)]
    a, b = _model(), _model()
    for bt in batches:
        a.train_step(bt)
    for i, bt in enumerate(batches):
        b.train_step(bt, batches[i + 1] if i + 1 < len(batches) else None)
    torch.cuda.synchronize()
    for x, y in zip(_state(a), _state(b)):
        assert torch.equal(x, y)


def test_lookahead_graph_ring_matches_eager_bitwise():
    gen = CriteoSynth(20000, device="cuda", seed=16)
    batches = [gen.batch(1024) for _ in range(4)]
    a, b = _model(), _model()
    order = [0, 1, 2, 3, 0, 1, 2]
    for i in order:
        a.train_step(batches[i])
    bufs = b.lookahead_graph_buffers(batches[0], 4)
    for dst, src in zip(bufs, batches):
        for d, s in ((dst.labels, src.labels), (dst.offsets, src.offsets), (dst.ids, src.ids)):
            d.copy_(s)
    losses = [b.train_step(bufs[i], bufs[(i + 1) % 4]).mean_loss() for i in order]
    torch.cuda.synchronize()
    for x, y in zip(_state(a), _state(b)):
        assert torch.equal(x, y)
    assert all(l == l for l in losses)


@pytest.mark.parametrize("dtype", [torch.bfloat16, K.FP8])
def test_stochastic_rounding_keeps_small_updates(dtype):
    """SGD steps far below half an ulp of the stored values: stochastic rounding (per-step
    device seed) follows the fp32 trajectory in expectation, round-to-nearest does not."""
    from fast_tffm_amd.models.table import FMTable

    rows, k, steps, lr = 4096, 64, 200, 1e-4
    opt = K.OptConfig("sgd", lr=lr)
    fp8 = dtype == K.FP8
    ends = {}
    for sr in (False, True):
        t = FMTable(rows, k, dtype=dtype, opt=opt, init=False, device="cuda")
        init = torch.full((rows, t.Kp), 0.75, device="cuda")
        if fp8:  # column 0 (= the row max) pins the per-row scale; the others sit at q = 224
            init.fill_(0.5)
            init[:, 0] = 1.0
            q, sc = K.quantize_fp8_rows(init)
            t.v.copy_(q)
            t.scale.copy_(sc)
        else:
            t.v.copy_(init.to(dtype))
        ctr = torch.zeros(1, dtype=torch.int32, device="cuda") if sr else None
        dd = K.dedup(torch.arange(rows, dtype=torch.int32, device="cuda"), key_bits=32, want_perm=True)
        grad = torch.ones((rows, t.Kp + 4), device="cuda")  # each step: v -= lr
        for _ in range(steps):
            if ctr is not None:
                ctr.add_(1)
            K.apply_rows(dd, grad, t.state, opt, t.Kp, sr_counter=ctr)
        cols = t.reference_rows()[:, 2:].double()  # factor columns (col 0 of reference rows is w)
        ends[sr] = cols.mean().item()
    start = 0.5 if fp8 else 0.75
    expect = start - steps * lr
    assert abs(ends[True] - expect) < 0.15 * steps * lr           # unbiased within noise
    assert abs(ends[False] - expect) > 0.4 * steps * lr           # nearest rounding drifts away


@pytest.mark.parametrize("B,maxf", [(131072, 39), (1000, 0), (777, 200), (64, 5), (1, 70), (3000, 1)])
def test_csr_rows_matches_torch(B, maxf):
    """csr_rows_kernel (a wave per 64 examples, shuffle search) vs repeat_interleave: example
    index and packed (example << bits | slot) code, with empty examples, examples longer than
    a wave and B not a multiple of 64."""
    g = torch.Generator().manual_seed(B + maxf)
    sizes = torch.randint(0, maxf + 1, (B,), generator=g, dtype=torch.int32)
    if maxf:
        sizes[:: 7] = 0
    offs = torch.zeros(B + 1, dtype=torch.int32)
    offs[1:] = torch.cumsum(sizes, 0)
    nnz = int(offs[-1])
    ex = torch.repeat_interleave(torch.arange(B, dtype=torch.int32), sizes)
    slot = torch.arange(nnz, dtype=torch.int32) - torch.repeat_interleave(offs[:-1], sizes)
    d = offs.cuda()
    torch.testing.assert_close(K.csr_rows(d, nnz=nnz).cpu(), ex, rtol=0, atol=0)
    bits = max(1, int(max(int(sizes.max()), 1) - 1).bit_length())
    torch.testing.assert_close(K.csr_rows(d, nnz=nnz, slot_bits=bits).cpu(), (ex << bits) | slot, rtol=0, atol=0)
