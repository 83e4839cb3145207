"""GPU libsvm tokenizer (hip/parse.hip) vs the CPU parser (reference FmParser grammar,
cc/fm_parser_op.cc:58-109): same CSR on supported syntax, CPU fallback otherwise."""

import os

import numpy as np
import pytest
import torch

from fast_tffm_amd.data.reader import NativeTextReader
from fast_tffm_amd.data.synthetic import write_libsvm
from fast_tffm_amd.ops import kernels as K
from fast_tffm_amd.ops import native

pytestmark = pytest.mark.gpu


def _lines_to_dev(lines):
    data = b"".join(l + b"\n" for l in lines)
    starts = np.zeros(len(lines) + 1, dtype=np.int64)
    np.cumsum([len(l) + 1 for l in lines], out=starts[1:])
    buf = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    return data, buf, torch.from_numpy(starts).cuda()


def _cpu(data, vocab, hashed):
    labels, sizes, ids, vals = native.cpu().parse_buffer(data, vocab, hashed, 2)
    offs = np.zeros(len(sizes) + 1, dtype=np.int64)
    np.cumsum(sizes, out=offs[1:])
    return labels, offs, ids, vals


def _check_same(lines, vocab, hashed=False):
    data, buf, ls = _lines_to_dev(lines)
    pg = K.parse_gpu(buf, ls, vocab, hashed)
    assert not pg.fallback
    labels, offs, ids, vals = _cpu(data, vocab, hashed)
    assert np.array_equal(pg.offsets.cpu().numpy(), offs)
    assert np.array_equal(pg.ids.cpu().numpy(), ids)
    assert np.array_equal(pg.labels.cpu().numpy(), labels)
    gv = pg.vals.cpu().numpy() if pg.vals is not None else np.ones(pg.nnz, np.float32)
    assert np.array_equal(gv, vals)
    assert pg.max_feats == (int(np.diff(offs).max()) if len(lines) else 0)
    return pg


def test_reference_fixture_lines():
    # fm_parser_op_test.py:7-15 semantic vectors (trailing space, decimal values)
    _check_same([b"1 1:0.5 2:0.6 ", b"0 3:0.7 4:0.8 5:0.9", b"1 6:0.1 7 8"], 10)


def test_synthetic_files_match(tmp_path):
    for with_values in (False, True):
        p = str(tmp_path / f"f{with_values}")
        write_libsvm(p, 3000, shape="criteo", vocab_size=1_000_000, seed=4, with_values=with_values)
        lines = open(p, "rb").read().splitlines()
        _check_same(lines, 1_000_000)


def test_reference_data(ref_data_dir):
    lines = open(os.path.join(ref_data_dir, "train_0"), "rb").read().splitlines()[:5000]
    _check_same(lines, 1_000_000)


def test_hashed_tokens():
    lines = [b"1 apple banana:2 c", b"0 apple", b"1 x:0.25 yy zzz:-1.5e-2"]
    pg = _check_same(lines, 10_007, hashed=True)
    assert pg.vals is not None


def test_labels_and_values_decimal_forms():
    _check_same([b"-1 1:1e-3 2:+2.5", b"0.25 3:.5 4:7.", b"+1 5:1E2 6:-0"], 10)


@pytest.mark.parametrize("line", [b"1  5", b"x 2", b"1 2:abc", b"1 20", b"1 +3", b"nan 1", b"1 2:3:4"])
def test_unsupported_or_bad_syntax_falls_back(line):
    _, buf, ls = _lines_to_dev([b"1 2 3", line])
    assert K.parse_gpu(buf, ls, 10).fallback


def test_reader_gpu_parse_equals_cpu_parse(tmp_path):
    files, wfiles = [], []
    for i in range(2):
        p, w = str(tmp_path / f"t{i}"), str(tmp_path / f"w{i}")
        write_libsvm(p, 2500, shape="criteo", vocab_size=100_000, seed=i, weights_path=w, with_values=i == 1)
        files.append(p)
        wfiles.append(w)
    kw = dict(vocab_size=100_000, num_epochs=2, seed=9, parse_threads=2)
    cpu = list(NativeTextReader(files, wfiles, 700, **kw))
    r = NativeTextReader(files, wfiles, 700, gpu_parse="cuda", **kw)
    gpu = list(r)
    assert r.fallbacks == 0 and len(cpu) == len(gpu)
    for a, b in zip(cpu, gpu):
        assert a.reader_pos == b.reader_pos and a.nnz == b.nnz and b.ids.is_cuda
        for x, y in ((a.labels, b.labels), (a.offsets, b.offsets), (a.ids, b.ids), (a.weights, b.weights)):
            assert torch.equal(x, y.cpu())
        ax = a.vals if a.vals is not None else torch.ones(a.nnz)
        bx = b.vals.cpu() if b.vals is not None else torch.ones(b.nnz)
        assert torch.equal(ax, bx)


def test_reader_cpu_parse_fed_to_device_equals_host_batches(tmp_path):
    """CPU parser + the C++ feeder (feed_device): the loader's CSR batches are copied to the device
    by the feeder thread; they equal the host batches of the same reader configuration, and list()
    holding every batch at once (more than the feeder's initial slots) still completes."""
    files, wfiles = [], []
    for i in range(2):
        p, w = str(tmp_path / f"t{i}"), str(tmp_path / f"w{i}")
        write_libsvm(p, 2500, shape="criteo", vocab_size=100_000, seed=i, weights_path=w, with_values=i == 0)
        files.append(p)
        wfiles.append(w)
    kw = dict(vocab_size=100_000, num_epochs=2, seed=3, parse_threads=2)
    host = list(NativeTextReader(files, wfiles, 600, **kw))
    r = NativeTextReader(files, wfiles, 600, feed_device="cuda", **kw)
    assert r.inline
    dev = list(r)
    assert len(host) == len(dev) > 6
    for a, b in zip(host, dev):
        assert a.reader_pos == b.reader_pos and a.nnz == b.nnz and b.ids.is_cuda and b.max_feats == a.max_feats
        for x, y in ((a.labels, b.labels), (a.offsets, b.offsets), (a.ids, b.ids), (a.weights, b.weights)):
            assert torch.equal(x, y.cpu())
        assert (a.vals is None) == (b.vals is None)
        if a.vals is not None:
            assert torch.equal(a.vals, b.vals.cpu())


def test_reader_gpu_parse_fallback_reports_errors(tmp_path):
    p = tmp_path / "bad"
    p.write_text("1 2 3\n1 2:xyz\n")
    with pytest.raises(ValueError, match="Invalid feature value"):
        list(NativeTextReader([str(p)], None, 4, vocab_size=10, gpu_parse="cuda"))


@pytest.mark.parametrize("mode", ["feed_device", "gpu_parse"])
def test_feeder_grows_slots_for_denser_batches(tmp_path, mode):
    """The feeder's device slots are sized from the files' heads; batches far denser than that
    (long lines after short ones) make it ask for larger ids / vals buffers instead of failing
    (ADVICE r3), and the batches still equal the host reader's."""
    p = tmp_path / "mixed"
    with open(p, "w") as f:
        for i in range(20000):
            f.write(f"{i % 2} {i % 97}\n")
        for i in range(600):
            f.write(f"{i % 2} " + " ".join(str((i * 7 + j) % 50000) for j in range(100)) + "\n")
    kw = dict(vocab_size=100_000, num_epochs=1, seed=5, parse_threads=2)
    host = list(NativeTextReader([str(p)], None, 256, **kw))
    r = NativeTextReader([str(p)], None, 256, **{mode: "cuda"}, **kw)
    dev = list(r)
    assert r.resizes > 0 and len(host) == len(dev)
    for a, b in zip(host, dev):
        assert a.reader_pos == b.reader_pos and a.nnz == b.nnz and b.ids.is_cuda
        for x, y in ((a.labels, b.labels), (a.offsets, b.offsets), (a.ids, b.ids)):
            assert torch.equal(x, y.cpu())
