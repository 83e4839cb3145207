"""HBM-resident training data (data/device_cache.py + hip/batch_gather.hip) on the GPU.

The device-gathered batches must equal the host binary loader's batches bit for bit
(same rows drawn, same CSR), and training from the device cache must give the same
losses as training from the text files."""

import contextlib
import io
import re

import numpy as np
import pytest
import torch

from fast_tffm_amd import cli
from fast_tffm_amd.data import bincache
from fast_tffm_amd.data.reader import NativeTextReader, ReaderState

pytestmark = pytest.mark.gpu

V = 50_000


def _write(path, n, seed, values=False):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for _ in range(n):
            k = int(rng.integers(0, 80))  # some rows longer than a wave
            toks = [str(j) + (f":{rng.uniform(0.1, 2):.3f}" if values else "") for j in rng.integers(0, V, k)]
            f.write(f"{int(rng.integers(0, 2))} " + " ".join(toks) + "\n")
    with open(path + ".w", "w") as f:
        for _ in range(n):
            f.write(f"{rng.uniform(0.5, 2):.4f}\n")


@pytest.fixture()
def caches(tmp_path):
    files = []
    for i, n in enumerate((1300, 700, 555)):
        files.append(str(tmp_path / f"t{i}"))
        _write(files[-1], n, i, values=(i == 2))
    return [p for p, _ in bincache.convert_files(files, [f + ".w" for f in files], str(tmp_path / "fmb"), V)]


def _collect(reader):
    out = []
    for b in reader:
        out.append([None if t is None else t.cpu().numpy().copy() for t in (b.labels, b.offsets, b.ids, b.vals,
                                                                              b.weights)] + [b.reader_pos, b.nnz])
    return out


@pytest.mark.parametrize("shuffle,rank,world", [(True, 0, 1), (False, 0, 1), (True, 1, 2)])
def test_device_gather_equals_host_batches(caches, shuffle, rank, world):
    kw = dict(vocab_size=V, num_epochs=2, shuffle=shuffle, seed=3, rank=rank, world=world)
    host = _collect(NativeTextReader(caches, None, 128, **kw))
    r = NativeTextReader(caches, None, 128, device_cache="cuda", **kw)
    assert r.dds is not None and r.dds.N == 1300 + 700 + 555
    dev = _collect(r)
    assert len(dev) == len(host) > 5
    for a, b in zip(dev, host):
        for x, y in zip(a[:5], b[:5]):
            assert (x is None) == (y is None)
            if x is not None:
                np.testing.assert_array_equal(x, y)
        assert a[5:] == b[5:]
    # resume from a position
    ep, cnt = host[4][5]
    res = _collect(NativeTextReader(caches, None, 128, device_cache="cuda", state=ReaderState(ep, cnt), **kw))
    assert len(res) == len(host) - 5 and all(np.array_equal(x[2], y[2]) for x, y in zip(res, host[5:]))


def test_train_from_device_cache_matches_text(tmp_path):
    d = tmp_path / "data"
    d.mkdir()
    for i in range(2):
        _write(str(d / f"train_{i}"), 2000, 10 + i)
    base = f"""[General]
vocabulary_size = {V}
vocabulary_block_num = 2
factor_num = 8
hash_feature_id = False
log_dir = {{log}}
device = cuda
[Train]
batch_size = 500
init_value_range = 0.01
factor_lambda = 0.0001
bias_lambda = 0.0001
epoch_num = 2
learning_rate = 0.05
adagrad.initial_accumulator = 0.1
save_steps = 100
loss_type = logistic
train_files = {{train}}
{{extra}}
[Predict]
predict_files =
"""
    cfg = tmp_path / "a.cfg"
    cfg.write_text(base.format(log=tmp_path / "la", train=f"{d}/train_?", extra=f"weight_files = {d}/train_?.w"))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert cli.main(["convert", str(cfg), "--out", str(tmp_path / "fmb")]) == 0
    cfg2 = tmp_path / "b.cfg"
    cfg2.write_text(base.format(log=tmp_path / "lb", train=f"{tmp_path}/fmb/*.fmb", extra="device_cache = true"))
    outs = []
    for c in (cfg, cfg2):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert cli.main(["train", str(c)]) == 0
        outs.append(buf.getvalue())
    assert "Training data resident on cuda" in outs[1]
    la, lb = (re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", o) for o in outs)
    assert len(la) == 16 and la == lb
    torch.cuda.synchronize()
