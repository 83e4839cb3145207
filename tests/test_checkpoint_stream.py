"""Streamed checkpoint shards (utils/checkpoint.py::write_safetensors_streamed / _iter_row_chunks).

A shard is written chunk by chunk and restored chunk by chunk, so host memory holds
one chunk, not the table (a 125M-row k=64 shard with Adagrad slots is ~65 GB).  The
tests force many tiny chunks and check: the file is a standard safetensors file
(the library's own loader reads it back bit-exactly), save -> restore is exact for
fp32 / bf16 tables with FTRL's two slots, and the global bias survives."""

import torch
from safetensors.torch import load_file

from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K
from fast_tffm_amd.utils import checkpoint as ckpt


def _model(dtype=torch.float32, opt="adagrad", gbias=False):
    cfg = FMConfig(vocabulary_size=1013, factor_num=10, loss_type="logistic", batch_size=64, seed=5, dtype=dtype,
                   global_bias=gbias, opt=K.OptConfig(opt, lr=0.1))
    return FactorizationMachine(cfg, device="cpu")


def test_streamed_file_is_standard_safetensors(tmp_path, monkeypatch):
    monkeypatch.setattr(ckpt, "CHUNK_BYTES", 300)
    m = _model()
    m.train_step(random_batch(64, 1013, max_feats=8, seed=0))
    path = ckpt.save_checkpoint(m, str(tmp_path / "log"), m.global_step)
    shard = [f for f in __import__("os").listdir(path) if f.endswith(".safetensors")][0]
    got = load_file(f"{path}/{shard}")
    want = ckpt._table_tensors(m.table)
    assert set(want) <= set(got)
    for k, v in want.items():
        assert got[k].dtype == v.dtype and torch.equal(got[k], v), k


def test_streamed_round_trip(tmp_path, monkeypatch):
    monkeypatch.setattr(ckpt, "CHUNK_BYTES", 500)
    for dtype, opt, gbias in ((torch.float32, "ftrl", True), (torch.bfloat16, "adagrad", False)):
        m = _model(dtype, opt, gbias)
        for s in range(3):
            m.train_step(random_batch(64, 1013, max_feats=8, seed=s))
        path = ckpt.save_checkpoint(m, str(tmp_path / f"log_{opt}"), m.global_step)
        m2 = _model(dtype, opt, gbias)
        ckpt.restore_checkpoint(m2, path)
        a, b = ckpt._table_tensors(m.table), ckpt._table_tensors(m2.table)
        assert a.keys() == b.keys()
        for k in a:
            assert torch.equal(a[k], b[k]), (opt, k)
        if gbias:
            assert torch.equal(m.gbias, m2.gbias) and torch.equal(m.gbias_s0, m2.gbias_s0)
