"""SavedModel export of the serving graph (utils/saved_model.py): protobuf structure and graph
semantics, checked without TensorFlow through the module's own decoder and numpy interpreter
(parity with TF's loader itself is unpinned: TF is not installable here)."""

import numpy as np
import pytest

from fast_tffm_amd.utils import saved_model as sm
from fast_tffm_amd.utils.tf_bundle import read_bundle


def _dense_score(blocks, line, K, bias=0.0):
    N = len(blocks)
    s1, s2, lin = np.zeros(K), 0.0, 0.0
    for t in line.split():
        i, v = t.split(":")
        i, v = int(i), float(v)
        row = blocks[i % N][i // N].astype(np.float64)
        lin += row[0] * v
        s1 += row[1:] * v
        s2 += ((row[1:] * v) ** 2).sum()
    return lin + 0.5 * ((s1 ** 2).sum() - s2) + bias


@pytest.mark.parametrize("N,bias", [(1, None), (3, None), (10, 0.25)])
def test_saved_model_graph_scores(tmp_path, N, bias):
    V, K = 200, 5
    rng = np.random.default_rng(N)
    blocks = [rng.standard_normal((V // N + 1, K + 1)).astype(np.float32) for _ in range(N)]
    files = sm.write_saved_model(str(tmp_path), blocks, V, K, global_bias=bias)
    assert [f.rsplit("/", 1)[1] for f in files] == ["saved_model.pb", "variables.index",
                                                     "variables.data-00000-of-00001"]
    got = read_bundle(str(tmp_path / "variables" / "variables"))
    assert sorted(got) == [f"vocab_block_{i}" for i in range(N)]
    info = sm.read_saved_model(str(tmp_path))
    ops = {op for op, _, _ in info["nodes"].values()}
    assert {"Placeholder", "StringSplit", "StringToNumber", "SparseToDense", "VariableV2", "RestoreV2",
            "Assign", "NoOp"} <= ops
    assert ("DynamicPartition" in ops) == (N > 1)
    assert info["producer"] == sm.GRAPH_PRODUCER
    for name, (op, inputs, attrs) in info["nodes"].items():  # every input names an existing node
        for i in inputs:
            assert i.lstrip("^").split(":")[0] in info["nodes"], (name, i)
        if op == "VariableV2":
            assert attrs["shape"] == [V // N + 1, K + 1]
    lines = ["1:1.0 5:0.5 7:2", "199:1", "", "3:1 3:1", "  0:0.25   42:-1.5 "]
    want = [_dense_score(blocks, ln, K, bias or 0.0) for ln in lines]
    np.testing.assert_allclose(sm.run_graph(str(tmp_path), lines), want, rtol=1e-5, atol=1e-5)
    # input of any shape is flattened (reference: tf.reshape(data_lines, [-1]))
    np.testing.assert_allclose(sm.run_graph(str(tmp_path), np.array(lines[:4]).reshape(2, 2)), want[:4],
                               rtol=1e-5, atol=1e-5)


def test_tensor_and_shape_protos_decode():
    for v in (np.arange(6, dtype=np.int32).reshape(2, 3), np.float32(0.5), np.array([-1, 2], np.int64)):
        back = sm._decode_tensor(sm.tensor_proto(v))
        assert back.dtype == np.asarray(v).dtype and np.array_equal(back, v)
    assert sm._decode_shape(sm.shape_proto([-1, 7])) == [-1, 7]
    assert sm._decode_shape(sm.shape_proto(None)) is None
    assert list(sm._decode_tensor(sm.tensor_proto(["a", "bc"]))) == [b"a", b"bc"]
