"""Hot-dictionary dedup (hip/hdedup.hip) against the onesweep radix-sort plan: every plan array
bitwise equal, whatever the dictionary holds.

Covered: Criteo-shaped batches with a dictionary from another batch (the pipeline's situation), from
the same batch, empty, and holding rows absent from the batch; uniform keys of several widths and
sizes (a dictionary of their repeated keys, tiny and odd sizes, one key); chunk lengths 1 / 7 / 32;
and the local training step end to end (losses and tables bitwise equal to FM_DEDUP=onesweep).
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


def _plan(monkeypatch, mode, keys, payload, key_bits, CH=32, hd=None):
    monkeypatch.setenv("FM_DEDUP", mode)
    n = keys.numel()
    ws = K.DedupWorkspace(max(n, 1), DEV, CH)
    dd = K.dedup(keys, ws=ws, key_bits=key_bits, ex_of_occ=payload, hot_dict=hd if mode == "hd" else None)
    torch.cuda.synchronize()
    U, C = int(dd.counts[0]), int(dd.counts[1])
    out = dict(U=U, C=C, skeys=dd.skeys[:n].clone(), perm=dd.perm[:n].clone(), uniq=dd.uniq[:U].clone(),
               seg_start=dd.seg_start[: U + 1].clone(), seg_chunk=dd.seg_chunk[: U + 1].clone(),
               chunk_start=dd.chunk_start[: C + 1].clone(), chunk_seg=dd.chunk_seg[:C].clone(),
               chunk_key=dd.chunk_key[:C].clone(), counts=dd.counts[:8].clone())
    return out, dd


def _same(a, b):
    assert a["U"] == b["U"] and a["C"] == b["C"], (a["U"], b["U"], a["C"], b["C"])
    for k in a:
        if k in ("U", "C"):
            continue
        if k == "counts":  # U, #chunks and the zeroed backward counters
            assert torch.equal(a[k][:3], b[k][:3]) and int(a[k][4]) == int(b[k][4]) == 0, (a[k], b[k])
            continue
        assert torch.equal(a[k], b[k]), k


def _dict_from(monkeypatch, keys, key_bits):
    """A dictionary rebuilt from the plan of ``keys``."""
    hd = K.HotDict(DEV, refresh=1)
    payload = torch.arange(keys.numel(), dtype=torch.int32, device=DEV)
    _plan(monkeypatch, "hd", keys, payload, key_bits, hd=hd)  # (rebuilt after this plan)
    torch.cuda.synchronize()
    hd.refresh = 10 ** 9  # frozen from here on
    return hd


def _check(monkeypatch, keys, key_bits, hd, CH=32):
    payload = torch.arange(keys.numel(), dtype=torch.int32, device=DEV) * 3 + 1
    ref, _ = _plan(monkeypatch, "onesweep", keys, payload, key_bits, CH)
    got, _ = _plan(monkeypatch, "hd", keys, payload, key_bits, CH, hd=hd)
    _same(got, ref)
    # the ground truth too: keys ascending, ties in input order, uniq = torch.unique
    k = keys.long()
    n = k.numel()
    order = torch.sort(k * (n + 1) + torch.arange(n, device=DEV)).indices
    assert torch.equal(got["perm"], payload[order])
    assert torch.equal(got["uniq"].long(), torch.unique(k))


def _criteo(seed, B=131072, vocab=125_000_000):
    return CriteoSynth(vocab, seed=seed, device=DEV).batch(B).ids.to(torch.int32)


def test_criteo_dict_from_other_batch(monkeypatch):
    hd = _dict_from(monkeypatch, _criteo(5), 27)
    assert int(hd.n) > 1000
    _check(monkeypatch, _criteo(6), 27, hd)


def test_criteo_dict_from_same_batch_and_chunk_lengths(monkeypatch):
    keys = _criteo(7, B=40000)
    hd = _dict_from(monkeypatch, keys, 27)
    for CH in (1, 7, 32):
        _check(monkeypatch, keys, 27, hd, CH=CH)


def test_empty_dictionary(monkeypatch):
    hd = K.HotDict(DEV, refresh=10 ** 9)
    hd.plans = 1  # never rebuilt: empty
    _check(monkeypatch, _criteo(8, B=20000), 27, hd)


def test_dictionary_rows_absent_from_batch(monkeypatch):
    hd = _dict_from(monkeypatch, _criteo(9, B=30000, vocab=1 << 20), 20)
    g = torch.Generator(device=DEV).manual_seed(1)
    keys = torch.randint(0, 1 << 20, (50000,), device=DEV, generator=g, dtype=torch.int64).to(torch.int32)
    _check(monkeypatch, keys, 20, hd)


@pytest.mark.parametrize("n,bits", [(1, 27), (7, 3), (1000, 16), (16383, 27), (16385, 20), (300_001, 31),
                                    (1_000_003, 27), (2_000_000, 12), (70_000, 1)])
def test_uniform_keys(monkeypatch, n, bits):
    g = torch.Generator(device=DEV).manual_seed(n)
    keys = torch.randint(0, 2 ** bits, (n,), device=DEV, generator=g, dtype=torch.int64).to(torch.int32)
    hd = _dict_from(monkeypatch, keys, bits)
    _check(monkeypatch, keys, bits, hd)


def test_single_key(monkeypatch):
    keys = torch.full((100_000,), 12345, dtype=torch.int32, device=DEV)
    hd = _dict_from(monkeypatch, keys, 27)
    assert int(hd.n) == 1
    _check(monkeypatch, keys, 27, hd)


def _train(monkeypatch, mode, steps=12):
    monkeypatch.setenv("FM_DEDUP", mode)
    monkeypatch.setenv("FM_HD_REFRESH", "3")
    cfg = FMConfig(vocabulary_size=4_000_000, factor_num=64, loss_type="logistic", batch_size=16384,
                   init_value_range=0.01, seed=7, opt=K.OptConfig("adagrad", lr=0.05), mode="local")
    m = FactorizationMachine(cfg, device=DEV)
    gen = CriteoSynth(cfg.vocabulary_size, seed=11, device=DEV)
    pool = [gen.batch(cfg.batch_size) for _ in range(4)]
    losses = []
    for i in range(steps):
        out = m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])
        losses.append(out.loss_sum.clone())
    out = m.train_step(pool[0])  # a step without lookahead (the side-stream dedup of _local_train_step)
    losses.append(out.loss_sum.clone())
    torch.cuda.synchronize()
    v, w = m.table.v.clone(), m.table.w.clone()
    m.close()
    return torch.stack(losses), v, w


def test_local_step_hd_equals_onesweep(monkeypatch):
    la, va, wa = _train(monkeypatch, "onesweep")
    lb, vb, wb = _train(monkeypatch, "hd")
    assert torch.equal(la, lb) and torch.equal(va, vb) and torch.equal(wa, wb)
