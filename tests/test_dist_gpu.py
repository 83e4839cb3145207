"""Multi-rank step executors on the GPU through RCCL at world size 1 (the
gpurun box has one MI355X): the sharded / replicated exchanges run their real
collectives (all_to_all_single, all_gather, all_reduce on device buffers) and
must reproduce the local single-GPU step.  World > 1 is covered on CPU with
gloo (test_distributed.py)."""

import os
import socket

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
@pytest.mark.parametrize("dense", [False, True])
def test_rccl_world1_matches_local(rccl_ctx, mode, dense, monkeypatch):
    if dense:  # MFMA backward rows (EMIT mode on the sharded path), forced on a small batch
        monkeypatch.setattr(K, "dense_min_for", lambda B, Kp, CH=32: 48)
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
