"""TF-Serving-compatible REST server over a serving export (CPU): request formats,
dynamic batching of concurrent requests, status / metadata, error handling."""

import json
import os
import threading
import urllib.error
import urllib.request

import numpy as np
import pytest
import torch

from fast_tffm_amd.serving import SIGNATURE, ServingModel, parse_serving_lines
from fast_tffm_amd.serving_server import FMServer

V, K, N = 500, 8, 3


def _export(tmp_path):
    d = tmp_path / "export"
    (d / "variables").mkdir(parents=True)
    g = np.random.default_rng(0)
    for i in range(N):
        rows = V // N + 1
        np.save(d / "variables" / f"vocab_block_{i}.npy", g.uniform(-0.3, 0.3, (rows, K + 1)).astype(np.float32))
    meta = dict(SIGNATURE, format="fast_tffm_amd/serving-v1", vocabulary_size=V, vocabulary_block_num=N,
                factor_num=K, hash_feature_id=False, loss_type="logistic", global_step=7, global_bias=None)
    (d / "saved_model.json").write_text(json.dumps(meta))
    return str(d)


def _lines(n, seed):
    g = np.random.default_rng(seed)
    return [" ".join(f"{int(i)}:{float(x):.3f}" for i, x in zip(g.integers(0, V, g.integers(1, 9)),
                                                                   g.uniform(0, 2, 9))) for _ in range(n)]


def _post(port, doc, path="/v1/models/fm:predict"):
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=json.dumps(doc).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return json.loads(r.read())


def _oracle(export, lines):
    """Dense fp64 FM score of the reference layout (block id % N, row id // N, col 0 = w)."""
    blocks = [np.load(os.path.join(export, "variables", f"vocab_block_{i}.npy")) for i in range(N)]
    out = []
    for ln in lines:
        lin, s1, s2 = 0.0, np.zeros(K), np.zeros(K)
        for tok in ln.split():
            i, x = tok.split(":")
            i, x = int(i), float(x)
            r = blocks[i % N][i // N].astype(np.float64)
            lin += x * r[0]
            s1 += x * r[1:]
            s2 += (x * r[1:]) ** 2
        out.append(lin + 0.5 * float((s1 ** 2 - s2).sum()))
    return np.array(out)


@pytest.fixture()
def server(tmp_path):
    exp = _export(tmp_path)
    srv = FMServer(exp, port=0, device="cpu", batch_timeout_ms=20).start()
    yield srv, exp
    srv.close()


def test_formats_and_values(server):
    srv, exp = server
    lines = _lines(20, 1)
    ref = _oracle(exp, lines)
    r = _post(srv.port, {"instances": lines})
    np.testing.assert_allclose(r["predictions"], ref, rtol=1e-5, atol=1e-5)
    r = _post(srv.port, {"signature_name": "serving_default", "inputs": {"data_lines": lines}})
    np.testing.assert_allclose(r["outputs"]["scores"], ref, rtol=1e-5, atol=1e-5)
    r = _post(srv.port, {"inputs": lines})
    np.testing.assert_allclose(r["outputs"], ref, rtol=1e-5, atol=1e-5)
    # same as the in-process predictor (saved_model_cli run equivalent)
    np.testing.assert_allclose(ServingModel.load(exp, "cpu").predict(lines), ref, rtol=1e-5, atol=1e-5)


def test_concurrent_requests_are_batched(server):
    srv, exp = server
    reqs = [_lines(5 + i, 100 + i) for i in range(12)]
    out = [None] * len(reqs)

    def go(i):
        out[i] = _post(srv.port, {"instances": reqs[i]})["predictions"]

    ths = [threading.Thread(target=go, args=(i,)) for i in range(len(reqs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for i, lines in enumerate(reqs):
        np.testing.assert_allclose(out[i], _oracle(exp, lines), rtol=1e-5, atol=1e-5)
    assert srv.batcher.requests == len(reqs) and srv.batcher.batches < len(reqs)


def test_status_metadata_and_errors(server):
    srv, _ = server
    with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/v1/models/fm", timeout=10) as r:
        st = json.loads(r.read())
    assert st["model_version_status"][0]["state"] == "AVAILABLE" and st["model_version_status"][0]["version"] == "7"
    with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/v1/models/fm/metadata", timeout=10) as r:
        md = json.loads(r.read())
    assert "serving_default" in md["metadata"]["signature_def"]["signature_def"]
    for bad in ({"instances": ["3 4:1"]}, {"instances": ["600:1"]}, {"foo": 1}, {"signature_name": "x", "inputs": []}):
        with pytest.raises(urllib.error.HTTPError) as e:
            _post(srv.port, bad)
        assert e.value.code == 400
    # a bad request in a coalesced batch does not fail the good ones
    assert len(_post(srv.port, {"instances": _lines(3, 5)})["predictions"]) == 3


def test_parse_serving_lines_whitespace_and_values():
    offs, ids, vals = parse_serving_lines(["  1:0.5   2:2 ", "3:1"], 10)
    assert offs.tolist() == [0, 2, 3] and ids.tolist() == [1, 2, 3]
    assert torch.allclose(vals, torch.tensor([0.5, 2.0, 1.0]))
    with pytest.raises(ValueError, match="id:val"):
        parse_serving_lines(["1:2 3"], 10)


@pytest.mark.gpu
def test_gpu_serving_matches_cpu(tmp_path):
    """GPU predict (GPU tokenizer behind a dummy label + fm_forward) == the CPU predictor;
    lines outside the tokenizer's subset (extra spaces) take the CPU parse; bad lines raise."""
    exp = _export(tmp_path)
    lines = _lines(300, 3) + ["  1:0.5   2:2 ", ""]
    cpu = ServingModel.load(exp, "cpu").predict(lines)
    gm = ServingModel.load(exp, "cuda")
    np.testing.assert_allclose(gm.predict(lines[:300]), cpu[:300], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(gm.predict(lines), cpu, rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError, match="id:val"):
        gm.predict(["1:2 3"])
