"""The bucket sort of the GPU dedup (hip/dedup.hip: stable MSD partition by the top key bits +
per-bucket LDS sort, rocPRIM segmented sort for oversize buckets) against rocPRIM's onesweep
radix sort (FM_DEDUP_SORT=onesweep, the round-2 path): every plan array bitwise equal.

Covered: Criteo-shaped batches (oversize buckets of very hot rows: the segmented fallback),
uniform keys, tiny and odd sizes, narrow and full key widths, a device count below the
capacity (the hot-row filter's kept count) and the local training step end to end.
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


def _plan(monkeypatch, algo, keys, payload, key_bits, n_dev=None, CH=32):
    monkeypatch.setenv("FM_DEDUP_SORT", algo)
    n = keys.numel() if n_dev is None else int(n_dev.item())
    if algo == "onesweep" and n_dev is not None:
        keys, payload = keys[:n], payload[:n]
        n_dev = None
    ws = K.DedupWorkspace(max(keys.numel(), 1), DEV, CH)
    dd = K.dedup(keys, ws=ws, key_bits=key_bits, ex_of_occ=payload, n_dev=n_dev)
    torch.cuda.synchronize()
    U, C = int(dd.counts[0]), int(dd.counts[1])
    return dict(U=U, C=C, skeys=dd.skeys[:n].clone(), perm=dd.perm[:n].clone(), uniq=dd.uniq[:U].clone(),
                seg_start=dd.seg_start[: U + 1].clone(), seg_chunk=dd.seg_chunk[: U + 1].clone(),
                chunk_start=dd.chunk_start[: C + 1].clone(), chunk_seg=dd.chunk_seg[:C].clone(),
                chunk_key=dd.chunk_key[:C].clone())


def _same(a, b):
    assert a["U"] == b["U"] and a["C"] == b["C"]
    for k in a:
        if k not in ("U", "C"):
            assert torch.equal(a[k], b[k]), k


def _check(monkeypatch, keys, key_bits, n_dev=None):
    payload = torch.arange(keys.numel(), dtype=torch.int32, device=DEV)
    ref = _plan(monkeypatch, "onesweep", keys, payload, key_bits, n_dev)
    got = _plan(monkeypatch, "bucket", keys, payload, key_bits, n_dev)
    _same(got, ref)
    n = keys.numel() if n_dev is None else int(n_dev.item())
    # the ground truth too: keys ascending, ties in input order, uniq = torch.unique
    k = keys[:n].long()
    order = torch.sort(k * (n + 1) + torch.arange(n, device=DEV)).indices
    assert torch.equal(got["perm"], order.to(torch.int32))
    assert torch.equal(got["uniq"].long(), torch.unique(k))


def test_criteo_batch_with_oversize_buckets(monkeypatch):
    b = CriteoSynth(125_000_000, seed=5, device=DEV).batch(131072)
    _check(monkeypatch, b.ids.to(torch.int32), 27)


@pytest.mark.parametrize("n,bits", [(1, 27), (7, 3), (1000, 16), (8191, 27), (8193, 20), (300_001, 31),
                                    (1_000_003, 27), (2_000_000, 12)])
def test_uniform_keys(monkeypatch, n, bits):
    g = torch.Generator(device=DEV).manual_seed(n)
    keys = torch.randint(0, 2 ** bits, (n,), device=DEV, generator=g, dtype=torch.int64).to(torch.int32)
    _check(monkeypatch, keys, bits)


def test_device_count_below_capacity(monkeypatch):
    g = torch.Generator(device=DEV).manual_seed(3)
    keys = torch.randint(0, 2 ** 24, (500_000,), device=DEV, generator=g, dtype=torch.int64).to(torch.int32)
    for n in (0, 1, 8192, 123_457, 500_000):
        _check(monkeypatch, keys, 24, n_dev=torch.tensor([n], dtype=torch.int32, device=DEV))


def _train(monkeypatch, algo, steps=10):
    monkeypatch.setenv("FM_DEDUP_SORT", algo)
    cfg = FMConfig(vocabulary_size=4_000_000, factor_num=64, loss_type="logistic", batch_size=16384,
                   init_value_range=0.01, seed=7, opt=K.OptConfig("adagrad", lr=0.05), mode="local")
    m = FactorizationMachine(cfg, device=DEV)
    gen = CriteoSynth(cfg.vocabulary_size, seed=11, device=DEV)
    pool = [gen.batch(cfg.batch_size) for _ in range(4)]
    losses = []
    for i in range(steps):
        out = m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])
        losses.append(out.loss_sum.clone())
    torch.cuda.synchronize()
    v, w = m.table.v.clone(), m.table.w.clone()
    m.close()
    return torch.stack(losses), v, w


def test_local_step_bucket_equals_onesweep(monkeypatch):
    la, va, wa = _train(monkeypatch, "onesweep")
    lb, vb, wb = _train(monkeypatch, "bucket")
    assert torch.equal(la, lb) and torch.equal(va, vb) and torch.equal(wa, wb)
