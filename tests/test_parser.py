"""libsvm parser + Hash64 parity.

Ports the semantic vectors of the reference's test/fm_parser_op_test.py:7-81
(testNoHash, testWithHash, testError) and adds the TF Hash64 vectors derived in
SURVEY.md §2.9 (tf.string_to_hash_bucket is not available here; the vectors
are pinned from the documented TF example ["Hello","TensorFlow","2.x"] % 3 ->
[2, 0, 1] and the survey's reconstruction for "1".."10" % 10000).
"""

import numpy as np
import pytest

from fast_tffm_amd.ops import native
from fast_tffm_amd.ops.fm_ops import fm_parser, string_to_hash_bucket

EXAMPLES = ["1 1:1 2:2 3:3 4:4", "-1 5:1 6:1 7:1 ", "1.0 8:0.1 9:0.2 10:0.3"]
VOCAB = 10000
TARGET_SIZES = [4, 3, 3]
TARGET_LABELS = [1, -1, 1.0]
TARGET_IDS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
TARGET_VALS = [1, 2, 3, 4, 1, 1, 1, 0.1, 0.2, 0.3]


def test_no_hash():
    labels, sizes, ids, vals = fm_parser(EXAMPLES, VOCAB)
    np.testing.assert_allclose(labels.numpy(), TARGET_LABELS)
    assert ids.tolist() == TARGET_IDS
    np.testing.assert_allclose(vals.numpy(), TARGET_VALS, rtol=1e-6)
    assert sizes.tolist() == TARGET_SIZES


def test_with_hash_matches_string_to_hash_bucket():
    labels, sizes, ids, vals = fm_parser(EXAMPLES, VOCAB, True)
    hashed = string_to_hash_bucket([str(x) for x in TARGET_IDS], VOCAB)
    np.testing.assert_allclose(labels.numpy(), TARGET_LABELS)
    assert sizes.tolist() == TARGET_SIZES
    assert ids.tolist() == hashed.tolist()
    np.testing.assert_allclose(vals.numpy(), TARGET_VALS, rtol=1e-6)


def test_hash64_vectors():
    assert string_to_hash_bucket(["Hello", "TensorFlow", "2.x"], 3).tolist() == [2, 0, 1]
    assert string_to_hash_bucket([str(i) for i in range(1, 11)], 10000).tolist() == [
        2333, 1362, 4535, 1205, 4140, 7902, 7642, 7211, 8813, 4343]
    # 8-byte block path and every tail length
    for s in ["", "a", "abcdefgh", "abcdefghi", "abcdefghijklmnopq"]:
        assert 0 <= native.cpu().hash64(s.encode()) < 2**64


@pytest.mark.parametrize("line,msg", [
    ("one 1:1 2:2 3:3 4:4", "Label could not be read in example: "),
    ("1 one:1 2:2 3:3 4:4", "Invalid format in example: "),
    ("1 1:one 2:2 3:3 4:4", "Invalid feature value. "),
    ("1 10000:1", r"Invalid feature id\. Should be in range \[0, vocabulary_size\)\."),
    ("1 -3:1", r"Invalid feature id\."),
    ("1 5:1\t6:1", "Invalid format in example: "),
])
def test_errors(line, msg):
    with pytest.raises(ValueError, match=msg):
        fm_parser([line], VOCAB)


def test_grammar_edge_cases():
    # trailing space accepted, missing features allowed, strtoll skips a second blank like the reference
    labels, sizes, ids, vals = fm_parser(["0 ", "2.5", "1 3  4:2"], VOCAB)
    assert sizes.tolist() == [0, 0, 2]
    assert ids.tolist() == [3, 4]
    assert vals.tolist() == [1.0, 2.0]
    np.testing.assert_allclose(labels.numpy(), [0, 2.5, 1])
    # hash mode: token ends at ':' and the value is parsed after it
    _, _, hid, hv = fm_parser(["1 abc:0.5 xyz"], VOCAB, True)
    assert hid.tolist() == string_to_hash_bucket(["abc", "xyz"], VOCAB).tolist()
    np.testing.assert_allclose(hv.numpy(), [0.5, 1.0])


def test_multithreaded_parse_equals_sequential():
    rng = np.random.default_rng(0)
    lines = []
    for i in range(20000):
        n = rng.integers(1, 30)
        feats = " ".join(f"{rng.integers(0, 99999)}:{rng.random():.4f}" for _ in range(n))
        lines.append(f"{rng.integers(0, 2)} {feats}")
    a = fm_parser(lines, 100000, threads=1)
    b = fm_parser(lines, 100000, threads=8)
    for x, y in zip(a, b):
        assert np.array_equal(x.numpy(), y.numpy())


def test_parse_buffer_crlf_and_weights():
    buf = b"1 1:1 2:2\r\n0 3:1\n"
    labels, sizes, ids, vals = native.cpu().parse_buffer(buf, 100, False, 1)
    assert sizes.tolist() == [2, 1] and ids.tolist() == [1, 2, 3]
    w = native.cpu().parse_floats([b"2\n", b"1.5", b" 3 "])
    assert w.tolist() == [2.0, 1.5, 3.0]
    with pytest.raises(ValueError):
        native.cpu().parse_floats([b"abc"])
