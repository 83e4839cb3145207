"""The production asynchronous schedule, checked for exactness on the GPU.

Everywhere else the GPU suite runs with FM_DEBUG_CHECKS=1 (tests/conftest.py): the kernel
wrappers then read index ranges back to the host before their launches, which serialises the host
against the compute stream and narrows the windows in which the side (lookahead / plan) streams
overlap it.  Here the checks are off, as in bench.py and training, and the multi-batch lookahead
pipelines -- whose plan-slot reuse is ordered only by events -- run for many steps over a small
pool of batches that they cycle through (the 3-slot rotation wraps several times):

* the local step with the depth-2 lookahead that the headline bench runs
  (``train_step(b, next, next2)``, models/fm.py ``_local_lookahead_step``) against plain steps,
  bit for bit, at B=4096 and at the bench's B=131072;
* the row-sharded step at world 1 with the depth-2 plan pipeline and early row exchange (self rows
  off, so the early exchange, dirty scan and patch really run) against the local step;
* the dense all-reduce data-parallel step (config 3) with its lookahead dedup against the local step.
"""

import os

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

POOL, STEPS = 4, 12


@pytest.fixture
def production(monkeypatch):
    """FM_DEBUG_CHECKS off for the test (no host syncs inside the kernel wrappers)."""
    was = K.debug_checks()
    K.set_debug_checks(False)
    monkeypatch.setenv("FM_DEBUG_CHECKS", "0")
    yield
    K.set_debug_checks(was)


def _cfg(V, k=64, dtype=torch.float32, mode="local", batch_size=4096, **kw):
    return FMConfig(vocabulary_size=V, factor_num=k, loss_type="logistic", init_value_range=0.05, seed=3,
                    opt=K.OptConfig("adagrad", lr=0.05), batch_size=batch_size, factor_lambda=0.01,
                    bias_lambda=0.01, dtype=dtype, mode=mode, **kw)


def _state(m):
    st = m.table.state
    return [x.clone() for x in (st.v, st.w, st.s0v, st.s0w) if x is not None]


@pytest.mark.parametrize("k,dtype", [(64, torch.float32), (16, torch.bfloat16), (128, K.FP8)])
def test_local_depth2_lookahead_bitwise(production, k, dtype):
    V = 40000
    gen = CriteoSynth(V, device="cuda", seed=61)
    pool = [gen.batch(4096) for _ in range(POOL)]
    plain = FactorizationMachine(_cfg(V, k, dtype), device="cuda")
    piped = FactorizationMachine(_cfg(V, k, dtype), device="cuda")
    lp, lq = [], []
    for i in range(STEPS):
        b = pool[i % POOL]
        lp.append(plain.train_step(b).loss_sum)
        lq.append(piped.train_step(b, pool[(i + 1) % POOL], pool[(i + 2) % POOL]).loss_sum)
    torch.cuda.synchronize()
    assert piped._lpending is not None and piped._lpending2 is not None  # the depth-2 pipeline ran
    for x, y in zip(lp, lq):
        assert torch.equal(x, y)
    for x, y in zip(_state(plain), _state(piped)):
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))


def test_local_depth2_lookahead_bitwise_bench_shape(production):
    """The same at the headline bench's batch (B=131072, k=64 fp32 + Adagrad; 10M rows instead of
    125M to keep two tables cheap): here the side-stream dedup of batch t+2 and the compute chain of
    batch t really overlap (a 4096-example plan finishes long before its slot is reused)."""
    V, B = 10_000_000, 131072
    gen = CriteoSynth(V, device="cuda", seed=64)
    pool = [gen.batch(B) for _ in range(POOL)]
    plain = FactorizationMachine(_cfg(V, batch_size=B), device="cuda")
    piped = FactorizationMachine(_cfg(V, batch_size=B), device="cuda")
    lp, lq = [], []
    for i in range(STEPS):
        b = pool[i % POOL]
        lp.append(plain.train_step(b).loss_sum)
        lq.append(piped.train_step(b, pool[(i + 1) % POOL], pool[(i + 2) % POOL]).loss_sum)
    torch.cuda.synchronize()
    assert piped._lpending is not None and piped._lpending2 is not None
    for x, y in zip(lp, lq):
        assert torch.equal(x, y)
    for x, y in zip(_state(plain), _state(piped)):
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))
    plain.close()
    piped.close()


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


@pytest.mark.parametrize("k,dtype", [(64, torch.float32), (16, torch.bfloat16)])
def test_shard_world1_depth2_early_rows_matches_local(production, rccl_ctx, monkeypatch, k, dtype):
    monkeypatch.setenv("FM_SELF_ROWS", "0")  # own rows through the exchange: early rows + patch run
    V = 40000
    gen = CriteoSynth(V, device="cuda", seed=62)
    pool = [gen.batch(4096) for _ in range(POOL)]
    loc = FactorizationMachine(_cfg(V, k, dtype), device="cuda")
    dm = FactorizationMachine(_cfg(V, k, dtype, mode="shard", prefetch_rows="on"), device="cuda", dist=rccl_ctx)
    for i in range(STEPS):
        b = pool[i % POOL]
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, pool[(i + 1) % POOL], pool[(i + 2) % POOL]).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1)), (i, l1, l2)
    torch.cuda.synchronize()
    assert dm._exchange.early_steps >= STEPS - 2
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-6)
    dm.close()


@pytest.mark.parametrize("dense", [False, True])
def test_dp_dense_lookahead_matches_local(production, rccl_ctx, dense, monkeypatch):
    if dense:  # the dense-buffer path of N > 1 at world 1 (else the world-1 local step)
        monkeypatch.setenv("FM_DP_W1_LOCAL", "0")
    V = 40000
    gen = CriteoSynth(V, device="cuda", seed=63)
    pool = [gen.batch(4096) for _ in range(POOL)]
    loc = FactorizationMachine(_cfg(V), device="cuda")
    dm = FactorizationMachine(_cfg(V, mode="dp_dense"), device="cuda", dist=rccl_ctx)
    for i in range(STEPS):
        b = pool[i % POOL]
        l1 = loc.train_step(b).mean_loss()
        l2 = dm.train_step(b, pool[(i + 1) % POOL], pool[(i + 2) % POOL]).mean_loss()
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l1)), (i, l1, l2)
    torch.cuda.synchronize()
    torch.testing.assert_close(dm.table.reference_rows(), loc.table.reference_rows(), rtol=1e-5, atol=1e-7)
    dm.close()

