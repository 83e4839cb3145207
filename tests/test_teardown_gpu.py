"""Executor teardown without the garbage collector (round-1 GC-time abort, commit 62c2bac).

Models with captured hipGraph rings and sharded exchanges with their own RCCL plan
communicator are dropped mid-run with a plain ``del`` -- no ``gc.collect()`` anywhere --
and the process then keeps training and shuts the process group down.  Helpers and
exchanges hold the model through weak proxies, so the last reference going away closes
the model at once (``FactorizationMachine.__del__`` -> ``close()``); ``dist.shutdown()``
closes whatever is still alive before destroying the groups."""


import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    from ports import free_port

    return free_port()


def _cfg(mode="auto"):
    return FMConfig(vocabulary_size=50_000, factor_num=64, loss_type="logistic", seed=5, batch_size=1024,
                    opt=K.OptConfig("adagrad", lr=0.05), mode=mode)


def _batches(n, dev):
    g = CriteoSynth(50_000, device=dev, seed=11)
    return [g.batch(1024) for _ in range(n)]


def test_dropped_models_release_without_gc(monkeypatch):
    from fast_tffm_amd.parallel import dist as fmdist

    dev = torch.device("cuda:0")
    batches = _batches(4, dev)
    # 1) a lookahead hipGraph ring, replayed, then dropped
    m = FactorizationMachine(_cfg(), device=dev)
    bufs = m.lookahead_graph_buffers(batches[0], 4)
    for dst, src in zip(bufs, batches):
        for d, s in ((dst.labels, src.labels), (dst.offsets, src.offsets), (dst.ids, src.ids)):
            d.copy_(s)
    for i in range(6):
        m.train_step(bufs[i % 4], bufs[(i + 1) % 4])
    del m, bufs
    # 2) a sharded exchange with a separate plan communicator (dual mode forced at world 1),
    #    pipelined (pending plans, early rows in flight), then dropped
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.setenv("FM_COMM_MODE", "dual")
    ctx = fmdist.init_distributed(backend="nccl", rank=0, world=1, device="cuda:0", force_pg=True)
    ms = FactorizationMachine(FMConfig(**{**_cfg("shard").__dict__, "prefetch_rows": "on"}), device=dev, dist=ctx)
    assert ms._exchange.comm_mode == "dual"
    for i in range(5):
        ms.train_step(batches[i % 4], batches[(i + 1) % 4], batches[(i + 2) % 4])
    del ms
    # 3) training continues in the same process, then the group is shut down
    m2 = FactorizationMachine(_cfg(), device=dev)
    out = m2.train_step(batches[0])
    torch.cuda.synchronize()
    assert out.mean_loss() == out.mean_loss()
    ms2 = FactorizationMachine(FMConfig(**{**_cfg("shard").__dict__}), device=dev, dist=ctx)
    ms2.train_step(batches[1], batches[2], batches[3])
    fmdist.shutdown()          # closes ms2 (still referenced) before destroying the groups
    assert ms2.closed
    with pytest.raises(RuntimeError):
        ms2.train_step(batches[1])
    out = m2.train_step(batches[1])   # local models keep working without a process group
    torch.cuda.synchronize()
    assert out.mean_loss() == out.mean_loss()
