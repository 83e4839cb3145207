"""Native training-data loader (csrc/cpu/loader.h) vs the reference input pipeline contract
(tffm/fm_model.py:34-126: per-epoch file shuffle, shuffle window of 4.5 B lines,
allow_smaller_final_batch, line-aligned weight files, one file per worker)."""

import collections

import numpy as np
import pytest

from fast_tffm_amd.data.reader import NativeTextReader, ReaderState, load_file_batch


def _write(tmp_path, name, lines):
    p = tmp_path / name
    p.write_text("".join(l + "\n" for l in lines))
    return str(p)


def _files(tmp_path, nfiles=3, per=57):
    """Line i of file f: label f, ids (f*1000+i, 7), weight f*1000+i (so each line is identifiable)."""
    data, wts = [], []
    for f in range(nfiles):
        lines = [f"{f} {f * 1000 + i} 7:{(i % 5) / 4:.2f}" for i in range(per)]
        data.append(_write(tmp_path, f"d{f}", lines))
        wts.append(_write(tmp_path, f"w{f}", [str(f * 1000 + i) for i in range(per)]))
    return data, wts


def _keys(b):
    """(first id of each line, weight) pairs of a batch."""
    offs = b.offsets.numpy()
    ids = b.ids.numpy()
    w = b.weights.numpy()
    return [(int(ids[offs[i]]), int(w[i])) for i in range(b.B)]


@pytest.mark.parametrize("shuffle", [True, False])
def test_every_line_once_per_epoch_and_weights_aligned(tmp_path, shuffle):
    data, wts = _files(tmp_path)
    r = NativeTextReader(data, wts, 10, vocab_size=10_000, num_epochs=2, shuffle=shuffle, seed=3, parse_threads=3)
    per_epoch = collections.defaultdict(list)
    sizes = collections.defaultdict(list)
    for b in r:
        e, _ = b.reader_pos
        keys = _keys(b)
        assert all(i == w for i, w in keys)  # weight line stays with its data line
        per_epoch[e] += [i for i, _ in keys]
        sizes[e].append(b.B)
        assert b.ids.dtype.is_floating_point is False and str(b.ids.dtype) == "torch.int32"
    expect = sorted(f * 1000 + i for f in range(3) for i in range(57))
    assert sorted(per_epoch[0]) == expect and sorted(per_epoch[1]) == expect
    assert sizes[0] == [10] * 17 + [1]  # allow_smaller_final_batch
    if not shuffle:
        assert per_epoch[0] == expect  # file order, line order
    else:
        assert per_epoch[0] != expect and per_epoch[0] != per_epoch[1]


def test_values_match_the_parser(tmp_path):
    data, wts = _files(tmp_path, nfiles=1, per=40)
    ref = load_file_batch(data, wts, 10_000, False, 2)
    b = next(iter(NativeTextReader(data, wts, 100, vocab_size=10_000, shuffle=False)))
    assert np.array_equal(b.offsets.numpy(), ref.offsets.numpy())
    assert np.array_equal(b.ids.numpy(), ref.ids.numpy())
    assert np.allclose(b.vals.numpy(), ref.vals.numpy()) and np.allclose(b.labels.numpy(), ref.labels.numpy())
    assert b.max_feats == 2


def test_unit_values_are_dropped(tmp_path):
    p = _write(tmp_path, "u", ["1 3 4", "0 5:1 6"])
    b = next(iter(NativeTextReader([p], None, 8, vocab_size=10, shuffle=False)))
    assert b.vals is None and b.weights is None and b.ids.tolist() == [3, 4, 5, 6]


def test_resume_skips_exactly(tmp_path):
    data, wts = _files(tmp_path)
    full = [(b.reader_pos, _keys(b)) for b in NativeTextReader(data, wts, 10, vocab_size=10_000, num_epochs=2,
                                                                seed=5)]
    for cut in (3, 18, 21):
        pos = full[cut - 1][0]
        st = ReaderState(*pos)
        rest = [(b.reader_pos, _keys(b)) for b in NativeTextReader(data, wts, 10, vocab_size=10_000, num_epochs=2,
                                                                    seed=5, state=st)]
        assert rest == full[cut:]


@pytest.mark.parametrize("nfiles", [3, 1])
def test_ranks_split_the_data(tmp_path, nfiles):
    """world 2: whole files per rank when there are enough files, else every other line."""
    data, wts = _files(tmp_path, nfiles=nfiles)
    seen = []
    for rank in range(2):
        ids = []
        for b in NativeTextReader(data, wts, 7, vocab_size=10_000, rank=rank, world=2, seed=1):
            ids += [i for i, _ in _keys(b)]
        seen.append(set(ids))
        assert len(ids) == len(set(ids))
    assert not (seen[0] & seen[1])
    if nfiles == 1:
        assert seen[0] | seen[1] == set(range(57))
    else:  # files shuffled per epoch, rank r takes files r, r+2, ...: all files of this epoch covered
        assert len(seen[0] | seen[1]) == 3 * 57


def test_parse_error_and_weight_mismatch(tmp_path):
    bad = _write(tmp_path, "bad", ["1 2 3", "x 4"])
    with pytest.raises(ValueError, match="Label could not be read in example: x 4"):
        list(NativeTextReader([bad], None, 4, vocab_size=10))
    bad_id = _write(tmp_path, "bad_id", ["1 2 30"])
    with pytest.raises(ValueError, match=r"Invalid feature id. Should be in range \[0, vocabulary_size\)"):
        list(NativeTextReader([bad_id], None, 4, vocab_size=10))
    d = _write(tmp_path, "d", ["1 2", "0 3"])
    w = _write(tmp_path, "w", ["1"])
    with pytest.raises(RuntimeError, match="1 lines but"):
        list(NativeTextReader([d], [w], 4, vocab_size=10))
    with pytest.raises(ValueError, match="do not match"):
        NativeTextReader([d], [w, w], 4, vocab_size=10)


def test_hashed_ids(tmp_path):
    from fast_tffm_amd.ops import native

    p = _write(tmp_path, "h", ["1 apple banana:2", "0 apple"])
    b = next(iter(NativeTextReader([p], None, 4, vocab_size=1000, hash_feature_id=True, shuffle=False)))
    h = native.cpu()
    labels, sizes, ids, vals = h.parse_lines([b"1 apple banana:2", b"0 apple"], 1000, True, 1)
    assert b.ids.tolist() == [int(x) for x in ids]
