"""Binary CSR caches (.fmb: csrc/cpu/bincsr.{h,cpp}, loader binary mode, data/bincache.py).

The contract: a cache yields exactly the batches its text file yields through the
native loader for the same seed -- shuffle window draws, file order, per-rank file /
line sharding, weights, values, hashed ids, exact resume -- and the loader refuses
caches that do not match the model (vocabulary, hashing) or are corrupt."""

import contextlib
import io
import os
import re

import numpy as np
import pytest

from fast_tffm_amd import cli
from fast_tffm_amd.data import bincache
from fast_tffm_amd.data.reader import NativeTextReader, ReaderState, TextBatchReader

V = 50_000


def _write(path, n, seed, values=False, hashed=False, empty_every=0):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for i in range(n):
            if empty_every and i % empty_every == 0:
                f.write("\n")
            k = int(rng.integers(0, 12))
            ids = rng.integers(0, V, k)
            toks = [(f"tok{j}" if hashed else str(j)) + (f":{rng.uniform(0.1, 2):.3f}" if values else "")
                    for j in ids]
            f.write(f"{int(rng.integers(0, 2))} " + " ".join(toks) + "\n")


def _weights(path, n, seed):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for _ in range(n):
            f.write(f"{rng.uniform(0.5, 2):.4f}\n")


def _batches(files, wfiles, **kw):
    r = NativeTextReader(files, wfiles, kw.pop("B", 97), vocab_size=V, parse_threads=3, **kw)
    out = []
    for b in r:
        out.append((b.labels.numpy().copy(), b.offsets.numpy().copy(), b.ids.numpy().copy(),
                    None if b.vals is None else b.vals.numpy().copy(),
                    None if b.weights is None else b.weights.numpy().copy(), b.reader_pos))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for u, v in zip(x[:5], y[:5]):
            if u is None or v is None:
                assert u is None and v is None
            else:
                np.testing.assert_array_equal(u, v)
        assert x[5] == y[5]


@pytest.fixture()
def data(tmp_path):
    files, wfiles = [], []
    for i, n in enumerate((700, 450, 333)):
        files.append(str(tmp_path / f"train_{i}"))
        wfiles.append(str(tmp_path / f"weight_{i}"))
        _write(files[-1], n, i, values=(i == 1))
        _weights(wfiles[-1], n, 10 + i)
    out = tmp_path / "fmb"
    caches = [p for p, _ in bincache.convert_files(files, wfiles, str(out), V, threads=3)]
    return files, wfiles, caches


@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("rank,world", [(0, 1), (1, 2), (2, 4)])
def test_cache_yields_the_text_batches(data, shuffle, rank, world):
    files, wfiles, caches = data
    assert all(bincache.is_bin_file(c) for c in caches) and not bincache.is_bin_file(files[0])
    kw = dict(num_epochs=2, shuffle=shuffle, seed=5, rank=rank, world=world)
    want = _batches(files, wfiles, **kw)
    got = _batches(caches, None, **kw)
    _same(got, want)
    if world == 1:
        assert any(b[3] is not None for b in got)  # file 1 carries non-unit values
    # fewer files than ranks: every world-th example of each file
    _same(_batches(caches[:1], None, **kw), _batches(files[:1], wfiles[:1], **kw))


def test_resume_and_hashing(tmp_path):
    f = str(tmp_path / "h")
    _write(f, 900, 3, hashed=True)
    c = str(tmp_path / "h.fmb")
    st = bincache.convert(f, c, V, hash_feature_id=True, threads=2, chunk_lines=100)  # many chunks
    assert st["examples"] == 900 and not st["has_vals"]
    kw = dict(num_epochs=3, seed=1, hash_feature_id=True, B=64)
    full = _batches([c], None, **kw)
    _same(full, _batches([f], None, **kw))
    assert all(b[3] is None for b in full)  # all values 1: no value array
    k = 17  # resume inside epoch 1
    ep, cnt = full[k - 1][5]
    _same(_batches([c], None, state=ReaderState(ep, cnt), **kw), full[k:])


def test_empty_lines_dropped(tmp_path):
    f = str(tmp_path / "e")
    _write(f, 300, 4, empty_every=7)
    st = bincache.convert(f, str(tmp_path / "e.fmb"), V)
    assert st["examples"] == 300
    _same(_batches([str(tmp_path / "e.fmb")], None, shuffle=False), _batches([f], None, shuffle=False))


def test_refusals(data, tmp_path):
    files, wfiles, caches = data
    with pytest.raises(Exception, match="vocabulary_size 50000"):
        list(NativeTextReader(caches, None, 10, vocab_size=V + 1))
    with pytest.raises(ValueError, match="already hold the weights"):
        NativeTextReader(caches, wfiles, 10, vocab_size=V)
    with pytest.raises(ValueError, match="mix"):
        NativeTextReader([caches[0], files[1]], None, 10, vocab_size=V)
    with pytest.raises(ValueError, match="native loader"):
        TextBatchReader(caches, None, 10, vocab_size=V)
    # truncated file
    raw = open(caches[0], "rb").read()
    bad = str(tmp_path / "trunc.fmb")
    open(bad, "wb").write(raw[: len(raw) - 40])
    with pytest.raises(Exception, match="truncated"):
        list(NativeTextReader([bad], None, 10, vocab_size=V))
    # an id outside the vocabulary must never reach the kernels
    hdr = np.frombuffer(raw[:64], dtype=np.int64)
    n, nnz = int(hdr[2]), int(hdr[3])
    ids_off = 64 + ((4 * n + 7) // 8) * 8 * 2 + 8 * (n + 1)  # labels, weights, offsets
    arr = bytearray(raw)
    arr[ids_off: ids_off + 4] = np.array([V + 3], np.int32).tobytes()
    open(bad, "wb").write(bytes(arr))
    assert nnz > 0
    with pytest.raises(Exception, match="outside"):
        list(NativeTextReader([bad], None, 10, vocab_size=V, shuffle=False))
    # a parse error names the line, like the text path
    txt = str(tmp_path / "bad.txt")
    open(txt, "w").write("1 3:1\nx 4\n")
    with pytest.raises(ValueError, match="Label could not be read"):
        bincache.convert(txt, str(tmp_path / "bad.fmb"), V)
    assert not os.path.exists(str(tmp_path / "bad.fmb")) and not os.path.exists(str(tmp_path / "bad.fmb.tmp"))


def test_cli_convert_then_train(tmp_path):
    d = tmp_path / "data"
    d.mkdir()
    for i in range(2):
        _write(str(d / f"train_{i}"), 1500, i)
        _weights(str(d / f"weight_{i}"), 1500, 20 + i)
    base = f"""[General]
vocabulary_size = {V}
vocabulary_block_num = 2
factor_num = 4
hash_feature_id = False
log_dir = {{log}}
device = cpu
[Train]
batch_size = 500
init_value_range = 0.01
factor_lambda = 0.0001
bias_lambda = 0.0001
epoch_num = 1
learning_rate = 0.05
adagrad.initial_accumulator = 0.1
save_steps = 100
loss_type = logistic
train_files = {{train}}
{{weights}}
[Predict]
predict_files =
"""
    cfg = tmp_path / "a.cfg"
    cfg.write_text(base.format(log=tmp_path / "log_t", train=f"{d}/train_*", weights=f"weight_files = {d}/weight_*"))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert cli.main(["convert", str(cfg), "--out", str(tmp_path / "fmb")]) == 0
    assert "Done converting" in buf.getvalue()
    cfg2 = tmp_path / "b.cfg"
    cfg2.write_text(base.format(log=tmp_path / "log_b", train=f"{tmp_path}/fmb/*.fmb", weights=""))
    outs = []
    for c in (cfg, cfg2):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert cli.main(["train", str(c)]) == 0
        outs.append(re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", buf.getvalue()))
    assert len(outs[0]) == 6 and outs[0] == outs[1]  # same batches -> same losses


def _host_gather(caches, rows):
    """Reference gather of global rows from the cache files (numpy, via the header layout)."""
    from fast_tffm_amd.data.device_cache import read_header

    parts = []
    for c in caches:
        h = read_header(c)
        mm = np.memmap(c, dtype=np.uint8, mode="r")
        off = np.frombuffer(mm, np.int64, h["n"] + 1, h["offsets"])
        parts.append((h, mm, off))
    labels, ids, vals, weights = [], [], [], []
    base = np.cumsum([0] + [p[0]["n"] for p in parts])
    for r in rows:
        fi = int(np.searchsorted(base, r, side="right") - 1)
        h, mm, off = parts[fi]
        i = int(r - base[fi])
        labels.append(np.frombuffer(mm, np.float32, 1, h["labels"] + 4 * i)[0])
        weights.append(np.frombuffer(mm, np.float32, 1, h["weights"] + 4 * i)[0] if h["weights"] >= 0 else 1.0)
        k = int(off[i + 1] - off[i])
        ids.append(np.frombuffer(mm, np.int32, k, h["ids"] + 4 * int(off[i])))
        vals.append(np.frombuffer(mm, np.float32, k, h["vals"] + 4 * int(off[i])) if h["vals"] >= 0
                    else np.ones(k, np.float32))
    return (np.array(labels, np.float32), np.concatenate(ids), np.concatenate(vals), np.array(weights, np.float32))


def test_rows_mode_names_the_binary_batches(data):
    """Rows mode (the device cache's host half) emits the rows whose data the binary mode copies."""
    from fast_tffm_amd.ops import native

    _, _, caches = data
    kw = dict(batch_size=97, vocab_size=V, shuffle=True, num_epochs=2, seed=5, threads=2, rank=0, world=1)
    La = native.cpu().TextLoader(caches, [], binary=True, **kw)
    Lr = native.cpu().TextLoader(caches, [], binary=True, rows=True, **kw)
    nb = 0
    while True:
        a, r = La.next(), Lr.next()
        if a is None:
            assert r is None
            break
        labels, offsets, ids, vals, weights, mf, ep, cnt = a
        rows, roffs, has_vals, rmf, rep, rcnt = r
        assert (ep, cnt, mf) == (rep, rcnt, rmf) and np.array_equal(offsets, roffs)
        assert has_vals == (vals is not None)
        hl, hi, hv, hw = _host_gather(caches, rows)
        np.testing.assert_array_equal(labels, hl)
        np.testing.assert_array_equal(ids, hi)
        np.testing.assert_array_equal(weights, hw)
        if vals is not None:
            np.testing.assert_array_equal(vals, hv)
        nb += 1
    assert nb > 10


def test_file_batch_from_caches_equals_text(data):
    """Validation / predict inputs: a cache loads as the same one-batch CSR as its text file."""
    from fast_tffm_amd.data.reader import load_file_batch

    files, wfiles, caches = data
    a = load_file_batch(files, wfiles, V, False, 2)
    b = load_file_batch(caches, None, V, False, 2)
    for x, y in ((a.labels, b.labels), (a.offsets, b.offsets), (a.ids, b.ids), (a.vals, b.vals),
                 (a.weights, b.weights)):
        assert x is not None and y is not None and np.array_equal(x.numpy(), y.numpy())
    assert (a.nnz, a.max_feats) == (b.nnz, b.max_feats)
    c = load_file_batch(caches[:1], None, V, False, 2)  # file 0: all values 1 -> no value array
    assert c.vals is None
    with pytest.raises(ValueError, match="already hold the weights"):
        load_file_batch(caches, wfiles, V, False)


def test_take_rank_slice():
    """trainer._take (rank-strided sub-batch for distributed predict / validation)."""
    import torch

    from fast_tffm_amd.data.synthetic import random_batch
    from fast_tffm_amd.trainer import _take

    b = random_batch(57, 1000, max_feats=9, seed=4)
    for idx in (torch.arange(1, 57, 3), torch.arange(0), torch.tensor([5])):
        t = _take(b, idx)
        o = b.offsets.long()
        want = [b.ids[int(o[i]): int(o[i + 1])] for i in idx]
        assert torch.equal(t.ids, torch.cat(want) if want else b.ids[:0])
        assert torch.equal(t.labels, b.labels[idx]) and t.B == idx.numel()
        if b.vals is not None:
            assert torch.equal(t.vals, torch.cat([b.vals[int(o[i]): int(o[i + 1])] for i in idx]) if want
                               else b.vals[:0])
