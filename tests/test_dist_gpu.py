"""Multi-rank step executors on the GPU through RCCL at world size 1 (the
gpurun box has one MI355X): the sharded / replicated exchanges run their real
collectives (all_to_all_single, all_gather, all_reduce on device buffers) and
must reproduce the local single-GPU step.  World > 1 is covered on CPU with
gloo (test_distributed.py)."""

import os

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    from ports import free_port

    return free_port()


@pytest.fixture(scope="module")
def rccl_ctx():
    from fast_tffm_amd.parallel import dist as fmdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    ctx = fmdist.init_distributed(backend="nccl", rank=0, world=1, device="cuda:0", force_pg=True)
    yield ctx
    fmdist.shutdown()


def _cfg(mode, V):
    return FMConfig(vocabulary_size=V, factor_num=64, loss_type="logistic", init_value_range=0.05, seed=3,
                    opt=K.OptConfig("adagrad", lr=0.05), batch_size=2048, factor_lambda=0.01, bias_lambda=0.01,
                    mode=mode)


@pytest.mark.parametrize("mode", ["shard", "dp", "dp_dense"])
@pytest.mark.parametrize("emit", [False, True])
def test_rccl_world1_matches_local(rccl_ctx, mode, emit, monkeypatch):
    if emit:  # the N > 1 compute path run at world 1 instead of the world-1 local step
        if mode == "shard":  # EMIT backward + exchange
            monkeypatch.setenv("FM_SHARD_W1_LOCAL", "0")
        elif mode == "dp_dense":  # dense gradient buffer + dense_apply
            monkeypatch.setenv("FM_DP_W1_LOCAL", "0")
        else:
            pytest.skip("dp has no separate world-1 path")
    V = 50000
    gen = CriteoSynth(V, device="cuda", seed=21)
    batches = [gen.batch(2048) for _ in range(3)]
    loc = FactorizationMachine(_cfg("local", V), device="cuda")
    dm = FactorizationMachine(_cfg(mode, V), device="cuda", dist=rccl_ctx)
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, batches[i + 1] if i + 1 < len(batches) else None).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1))
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-7)
    ev = gen.batch(512)
    torch.testing.assert_close(dm.predict(ev), loc.predict(ev), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, K.FP8])
@pytest.mark.parametrize("W", [2, 5, 8])
def test_apply_runs_matches_sorted_apply(dtype, W):
    """Owner-side run-merge update (cross-run match + leader apply) == sort-based grouping.

    W source ranks each send an ascending run of distinct local rows (overlapping
    across runs, some empty); both paths must sum each row's gradients in rank
    order and apply one Adagrad step."""
    from fast_tffm_amd.models.table import FMTable

    g = torch.Generator().manual_seed(W)
    rows, k = 5000, 64
    opt = K.OptConfig("adagrad", lr=0.05)
    runs = []
    for q in range(W):
        n = 0 if q == 1 else int(torch.randint(200, 3000, (1,), generator=g))
        runs.append(torch.randperm(rows, generator=g)[:n].sort().values)
    req = torch.cat(runs).to(torch.int32).cuda()
    splits = [int(r.numel()) for r in runs]
    R = req.numel()
    tabs = [FMTable(rows, k, dtype=dtype, opt=opt, init_range=0.05, seed=7, device="cuda") for _ in range(2)]
    Kp = tabs[0].Kp
    grad = torch.randn((R, Kp + 4), generator=g).cuda()
    dd = K.dedup(req, key_bits=32, want_perm=True)
    K.apply_rows(dd, grad, tabs[0].state, opt, Kp)
    off = torch.tensor([0] + list(torch.tensor(splits).cumsum(0)), dtype=torch.int32, device="cuda")
    match = torch.empty(R * W, dtype=torch.int32, device="cuda")
    K.apply_runs(req, off, splits, grad, tabs[1].state, opt, Kp, match=match)
    torch.cuda.synchronize()
    for a, b in zip((tabs[0].v, tabs[0].w, tabs[0].s0v, tabs[0].s0w), (tabs[1].v, tabs[1].w, tabs[1].s0v, tabs[1].s0w)):
        assert torch.equal(a.float(), b.float())


@pytest.mark.parametrize("dtype,k", [(torch.bfloat16, 16), (K.FP8, 128), (torch.bfloat16, 64)])
def test_rccl_world1_shard_storage_wire_matches_local(rccl_ctx, dtype, k):
    """bf16 / fp8 tables cross the exchange as their stored bits: the sharded step equals the local one."""
    V = 50000
    gen = CriteoSynth(V, device="cuda", seed=22)
    batches = [gen.batch(2048) for _ in range(3)]

    def cfg(mode):
        return FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=3,
                        opt=K.OptConfig("ftrl", lr=0.05, l1=0.001, l2=0.001, beta=1.0), batch_size=2048,
                        factor_lambda=0.01, bias_lambda=0.01, mode=mode, dtype=dtype)

    loc = FactorizationMachine(cfg("local"), device="cuda")
    dm = FactorizationMachine(cfg("shard"), device="cuda", dist=rccl_ctx)
    assert dm._exchange.wire.dtype == dtype
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, batches[i + 1] if i + 1 < len(batches) else None).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1))
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-6)


def test_rccl_world1_shard_bf16_wire_close_to_fp32(rccl_ctx):
    """comm_dtype=bf16 on an fp32 table: rows are rounded for transport only (master rows stay fp32)."""
    V = 50000
    gen = CriteoSynth(V, device="cuda", seed=23)
    batches = [gen.batch(2048) for _ in range(3)]
    loc = FactorizationMachine(_cfg("local", V), device="cuda")
    c = _cfg("shard", V)
    c.comm_dtype = "bf16"
    dm = FactorizationMachine(c, device="cuda", dist=rccl_ctx)
    assert dm._exchange.wire.dtype == torch.bfloat16 and dm.table.v.dtype == torch.float32
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, batches[i + 1] if i + 1 < len(batches) else None).mean_loss()
        assert abs(l1 - l2) <= 2e-3 * max(1.0, abs(l1))
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("mb", [2, 3])
def test_rccl_world1_shard_microbatches_match_local(rccl_ctx, mb):
    """The micro-batched sharded step (parts with their own dedup, 2W owner runs) == the local step."""
    V = 50000
    gen = CriteoSynth(V, device="cuda", seed=24)
    batches = [gen.batch(2048) for _ in range(3)]
    loc = FactorizationMachine(_cfg("local", V), device="cuda")
    c = _cfg("shard", V)
    c.microbatches = mb
    dm = FactorizationMachine(c, device="cuda", dist=rccl_ctx)
    assert dm._exchange.nparts == mb
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, batches[i + 1] if i + 1 < len(batches) else None).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1))
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-6)
    ev = gen.batch(512)
    torch.testing.assert_close(dm.predict(ev), loc.predict(ev), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("self_rows", ["0", "1"])
@pytest.mark.parametrize("depth", [1, 2])
@pytest.mark.parametrize("dtype,k", [(torch.float32, 64), (torch.bfloat16, 16), (K.FP8, 128)])
def test_rccl_world1_early_exchange_matches_local(rccl_ctx, dtype, k, depth, self_rows, monkeypatch):
    """Early row exchange + dirty-row patch (prefetch_rows=on) is exact: every step equals the
    local step, though rows shared by consecutive batches are read before the update lands.
    FM_SELF_ROWS=0 sends the rank's own rows through the exchange (the early machinery then
    runs at world 1); with self rows every request is the rank's own and nothing is exchanged."""
    monkeypatch.setenv("FM_SELF_ROWS", self_rows)
    V = 20000
    gen = CriteoSynth(V, device="cuda", seed=25)
    batches = [gen.batch(2048) for _ in range(6)]

    def cfg(mode):
        return FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=3,
                        opt=K.OptConfig("adagrad", lr=0.05), batch_size=2048, factor_lambda=0.01,
                        bias_lambda=0.01, mode=mode, dtype=dtype, prefetch_rows="on")

    loc = FactorizationMachine(cfg("local"), device="cuda")
    dm = FactorizationMachine(cfg("shard"), device="cuda", dist=rccl_ctx)
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        nb = batches[i + 1] if i + 1 < len(batches) else None
        nb2 = batches[i + 2] if depth == 2 and i + 2 < len(batches) else None
        l2 = dm.train_step(b, nb, nb2).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1)), (i, l1, l2)
    torch.cuda.synchronize()
    assert dm._exchange.early_steps == (len(batches) - 1 if self_rows == "0" else 0)
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-6)


def _self_rows_env(monkeypatch, self_rows: str) -> None:
    """"0": no self rows (every row through the wire); "1": self rows (at world 1 the step then runs
    the local kernels); "emit": self rows on the EMIT path of world > 1 (FM_SHARD_W1_LOCAL=0)."""
    monkeypatch.setenv("FM_SELF_ROWS", "0" if self_rows == "0" else "1")
    if self_rows == "emit":
        monkeypatch.setenv("FM_SHARD_W1_LOCAL", "0")


@pytest.mark.parametrize("self_rows", ["0", "1", "emit"])
@pytest.mark.parametrize("dtype,k", [(torch.float32, 64), (torch.bfloat16, 16), (K.FP8, 128)])
def test_rccl_world1_split_backward_matches_local(rccl_ctx, dtype, k, self_rows, monkeypatch):
    """Backward split into every owner's first / second half of rows (overlap_grads=on, with
    the early row exchange) reduces exactly what the one-piece backward does (self rows: both
    pieces update their rows in place)."""
    _self_rows_env(monkeypatch, self_rows)
    V = 20000
    gen = CriteoSynth(V, device="cuda", seed=26)
    batches = [gen.batch(2048) for _ in range(5)]

    def cfg(mode):
        return FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=3,
                        opt=K.OptConfig("adagrad", lr=0.05), batch_size=2048, factor_lambda=0.01,
                        bias_lambda=0.01, mode=mode, dtype=dtype, prefetch_rows="on", overlap_grads="on")

    loc = FactorizationMachine(cfg("local"), device="cuda")
    dm = FactorizationMachine(cfg("shard"), device="cuda", dist=rccl_ctx)
    assert dm._exchange.overlap_grads
    for i, b in enumerate(batches):
        l1 = loc.train_step(b).mean_loss()
        nb = batches[i + 1] if i + 1 < len(batches) else None
        nb2 = batches[i + 2] if i + 2 < len(batches) else None
        l2 = dm.train_step(b, nb, nb2).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1)), (i, l1, l2)
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("self_rows", ["0", "1", "emit"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rccl_world1_pipelined_shard_step_is_bitwise_deterministic(rccl_ctx, dtype, self_rows, monkeypatch):
    """Race detection for the sharded pipeline: with the side-stream plan two
    batches ahead, the early row exchange + patches and the split backward all on, two runs
    of the same batches leave bit-identical tables (bf16 with stochastic rounding too)."""
    _self_rows_env(monkeypatch, self_rows)
    V = 20000
    gen = CriteoSynth(V, device="cuda", seed=27)
    batches = [gen.batch(4096) for _ in range(6)]

    def run():
        cfg = FMConfig(vocabulary_size=V, factor_num=64, loss_type="logistic", init_value_range=0.05, seed=3,
                       opt=K.OptConfig("adagrad", lr=0.05), batch_size=4096, factor_lambda=0.01, bias_lambda=0.01,
                       mode="shard", dtype=dtype, prefetch_rows="on", overlap_grads="on")
        m = FactorizationMachine(cfg, device="cuda", dist=rccl_ctx)
        losses = []
        for i, b in enumerate(batches):
            nb = batches[i + 1] if i + 1 < len(batches) else None
            nb2 = batches[i + 2] if i + 2 < len(batches) else None
            losses.append(m.train_step(b, nb, nb2).mean_loss())
        torch.cuda.synchronize()
        return m.table.reference_rows().cpu(), m.table.s0v.cpu().clone(), losses

    a, b = run(), run()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and a[2] == b[2]


@pytest.mark.parametrize("k,dtype,prefetch", [(64, torch.float32, "on"), (16, torch.bfloat16, "off"),
                                               (128, torch.float8_e4m3fn, "on")])
def test_rccl_world1_segment_lookup_bitwise(rccl_ctx, k, dtype, prefetch, monkeypatch):
    """The sharded forward's key -> segment bucket index (K.seg_index, FM_SEG_LOOKUP=1) finds
    exactly the segments of the dedup's inverse map: same table bits, same predictions."""
    import dataclasses

    V = 60000
    gen = CriteoSynth(V, device="cuda", seed=29)
    batches = [gen.batch(2048) for _ in range(4)]
    ev = gen.batch(777)
    res, preds = [], []
    for f in ("0", "1"):
        monkeypatch.setenv("FM_SEG_LOOKUP", f)
        cfg = dataclasses.replace(_cfg("shard", V), factor_num=k, dtype=dtype, prefetch_rows=prefetch)
        dm = FactorizationMachine(cfg, device="cuda", dist=rccl_ctx)
        for i, b in enumerate(batches):
            dm.train_step(b, batches[i + 1] if i + 1 < len(batches) else None,
                          batches[i + 2] if i + 2 < len(batches) else None)
        torch.cuda.synchronize()
        st = dm.table.state
        res.append([x.clone() for x in (st.v, st.w, st.s0v, st.s0w)])
        preds.append(dm.predict(ev).clone())
        dm.close()
    for x, y in zip(*res):
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))
    assert torch.equal(preds[0], preds[1])


def test_seg_index_matches_inverse_map():
    """Bucket index lookup == inverse map for every occurrence (keys with dense and sparse buckets)."""
    gen = CriteoSynth(1 << 20, device="cuda", seed=31)
    b = gen.batch(4096)
    keys = b.ids.int().contiguous()
    dd = K.dedup(keys, key_bits=20, ex_of_occ=K.csr_rows(b.offsets), want_inv=True)
    si = K.seg_index(dd, 20)
    torch.cuda.synchronize()
    U = dd.sync()
    uniq = dd.uniq[:U].long()
    bkt = keys.long() >> si.shift
    lo, hi = si.idx[bkt].long(), si.idx[bkt + 1].long()
    # the key's segment lies in [lo, hi) and is its position in the sorted keys
    seg = torch.searchsorted(uniq, keys.long())
    assert bool(((seg >= lo) & (seg < hi)).all())
    assert torch.equal(seg.int(), dd.inv[: keys.numel()])
