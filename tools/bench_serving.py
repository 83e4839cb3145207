#!/usr/bin/env python3
"""Serving throughput: in-process ServingModel.predict at several batch sizes and the
HTTP server (TF-Serving REST API, dynamic batching) under concurrent clients.

usage: python tools/bench_serving.py [--vocab V] [--k K] [--device cuda|cpu]
"""

import argparse
import json
import os
import sys
import tempfile
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fast_tffm_amd.serving import SIGNATURE, ServingModel  # noqa: E402
from fast_tffm_amd.serving_server import FMServer  # noqa: E402


def make_export(d, V, K, N=8):
    os.makedirs(os.path.join(d, "variables"))
    g = np.random.default_rng(0)
    for i in range(N):
        np.save(os.path.join(d, "variables", f"vocab_block_{i}.npy"),
                g.uniform(-0.05, 0.05, (V // N + 1, K + 1)).astype(np.float32))
    meta = dict(SIGNATURE, format="fast_tffm_amd/serving-v1", vocabulary_size=V, vocabulary_block_num=N,
                factor_num=K, hash_feature_id=False, loss_type="logistic", global_step=1, global_bias=None)
    with open(os.path.join(d, "saved_model.json"), "w") as f:
        json.dump(meta, f)


def lines(n, V, seed=0):
    g = np.random.default_rng(seed)
    ids = g.integers(0, V, (n, 39))
    return [" ".join(f"{i}:1" for i in row) for row in ids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--lines-per-request", type=int, default=256)
    ap.add_argument("--requests", type=int, default=40, help="per client")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        exp = os.path.join(td, "export")
        make_export(exp, a.vocab, a.k)
        m = ServingModel.load(exp, a.device)
        for bs in (256, 4096, 65536):
            ls = lines(bs, a.vocab, bs)
            m.predict(ls)
            t = time.perf_counter()
            reps = max(1, 200000 // bs)
            for _ in range(reps):
                m.predict(ls)
            dt = time.perf_counter() - t
            print(f"predict batch {bs:6d}: {reps * bs / dt / 1e6:6.3f} M lines/s  ({dt / reps * 1e3:.2f} ms/call)",
                  flush=True)
        srv = FMServer(exp, port=0, device=a.device, batch_timeout_ms=1.0).start()
        body = json.dumps({"instances": lines(a.lines_per_request, a.vocab, 7)}).encode()

        def client():
            for _ in range(a.requests):
                req = urllib.request.Request(f"http://127.0.0.1:{srv.port}/v1/models/fm:predict", data=body,
                                             headers={"Content-Type": "application/json"})
                with urllib.request.urlopen(req, timeout=60) as r:
                    r.read()

        t = time.perf_counter()
        ths = [threading.Thread(target=client) for _ in range(a.clients)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t
        n = a.clients * a.requests
        print(f"http {a.clients} clients x {a.requests} req x {a.lines_per_request} lines: {n / dt:8.1f} req/s, "
              f"{n * a.lines_per_request / dt / 1e6:.3f} M lines/s, {srv.batcher.batches} model calls", flush=True)
        srv.close()


if __name__ == "__main__":
    main()
