"""Online serving of a ``run.py generate`` export over HTTP, TF-Serving REST compatible.

The reference exports a SavedModel (signature ``serving_default``: ``data_lines``
-> ``scores``, run_tffm.py:93-120) for TensorFlow Serving.  This module serves
the same signature from the native kernels:

* ``GET  /v1/models/<name>``             model status (version = global step)
* ``GET  /v1/models/<name>/metadata``    signature definition
* ``POST /v1/models/<name>:predict``     ``{"instances": [line, ...]}`` ->
  ``{"predictions": [score, ...]}`` (row format), or ``{"inputs": {"data_lines":
  [...]}}`` / ``{"inputs": [...]}`` -> ``{"outputs": {"scores": [...]}}`` /
  ``{"outputs": [...]}`` (columnar format); errors -> HTTP 400 ``{"error": ...}``.

Concurrent requests are coalesced by a dynamic batcher: one thread collects the
pending requests' lines (up to ``max_batch`` lines or ``batch_timeout_ms``
after the first one) and scores them with ONE forward launch on the device
(ServingModel.predict), so GPU serving throughput scales with concurrency
instead of paying a kernel launch + host sync per request.

    python -m fast_tffm_amd.serving_server --dir EXPORT --port 8501 [--model-name fm]
"""

from __future__ import annotations

import argparse
import json
import queue
import sys
import threading
import time
from concurrent.futures import Future
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from .serving import SIGNATURE, ServingModel


class DynamicBatcher:
    """Coalesces concurrent predict calls into one model invocation."""

    def __init__(self, model: ServingModel, max_batch: int = 65536, timeout_ms: float = 2.0):
        self.model = model
        self.max_batch = max(1, int(max_batch))
        self.timeout = max(0.0, timeout_ms) / 1000.0
        self.q: queue.Queue = queue.Queue()
        self.batches = 0           # model invocations (for tests / metrics)
        self.requests = 0
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, name="fm-batcher", daemon=True)
        self._th.start()

    def submit(self, lines: list) -> Future:
        fut: Future = Future()
        self.q.put((lines, fut))
        return fut

    def close(self) -> None:
        self._stop.set()
        self.q.put(None)
        self._th.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.is_set():
            item = self.q.get()
            if item is None:
                return
            pending = [item]
            n = len(item[0])
            deadline = time.monotonic() + self.timeout
            while n < self.max_batch:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    nxt = self.q.get(timeout=left)
                except queue.Empty:
                    break
                if nxt is None:
                    self._stop.set()
                    break
                pending.append(nxt)
                n += len(nxt[0])
            self._score(pending)

    def _score(self, pending) -> None:
        lines = [ln for ls, _ in pending for ln in ls]
        try:
            scores = self.model.predict(lines) if lines else np.zeros(0, np.float32)
        except Exception:  # noqa: BLE001 -- isolate the bad request(s): score them one by one
            for ls, fut in pending:
                try:
                    fut.set_result(self.model.predict(ls) if ls else np.zeros(0, np.float32))
                except Exception as e:  # noqa: BLE001
                    fut.set_exception(e)
            return
        self.batches += 1
        self.requests += len(pending)
        o = 0
        for ls, fut in pending:
            fut.set_result(scores[o: o + len(ls)])
            o += len(ls)


def _lines_from_request(doc) -> tuple[list, str]:
    """(lines, format) from a TF-Serving predict request body."""
    if not isinstance(doc, dict):
        raise ValueError("request body must be a JSON object")
    if "instances" in doc:
        inst = doc["instances"]
        lines = [x["data_lines"] if isinstance(x, dict) else x for x in inst]
        return lines, "row"
    if "inputs" in doc:
        inp = doc["inputs"]
        if isinstance(inp, dict):
            if "data_lines" not in inp:
                raise ValueError("inputs must name data_lines")
            return list(np.asarray(inp["data_lines"]).reshape(-1)), "col_named"
        return list(np.asarray(inp).reshape(-1)), "col"
    raise ValueError("request needs 'instances' or 'inputs'")


def make_handler(batcher: DynamicBatcher, model_name: str, meta: dict):
    base = f"/v1/models/{model_name}"

    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # quiet
            pass

        def _send(self, code: int, doc) -> None:
            body = json.dumps(doc).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):  # noqa: N802
            path = self.path.rstrip("/")
            if path in (base, base + "/versions/" + str(meta.get("global_step", 0))):
                self._send(200, {"model_version_status": [{
                    "version": str(meta.get("global_step", 0)), "state": "AVAILABLE",
                    "status": {"error_code": "OK", "error_message": ""}}]})
            elif path == base + "/metadata":
                self._send(200, {"model_spec": {"name": model_name, "version": str(meta.get("global_step", 0))},
                                 "metadata": {"signature_def": {"signature_def": {
                                     SIGNATURE["signature_def"]: {"inputs": SIGNATURE["inputs"],
                                                                  "outputs": SIGNATURE["outputs"],
                                                                  "method_name": SIGNATURE["method_name"]}}}}})
            else:
                self._send(404, {"error": f"unknown path {self.path}"})

        def do_POST(self):  # noqa: N802
            if self.path.rstrip("/") not in (base + ":predict",):
                self._send(404, {"error": f"unknown path {self.path}"})
                return
            try:
                n = int(self.headers.get("Content-Length", "0"))
                doc = json.loads(self.rfile.read(n) or b"{}")
                sig = doc.get("signature_name", SIGNATURE["signature_def"]) if isinstance(doc, dict) else None
                if sig != SIGNATURE["signature_def"]:
                    raise ValueError(f"unknown signature {sig!r}")
                lines, fmt = _lines_from_request(doc)
                scores = batcher.submit(lines).result(timeout=60).tolist()
            except Exception as e:  # noqa: BLE001
                self._send(400, {"error": str(e)})
                return
            if fmt == "row":
                self._send(200, {"predictions": scores})
            elif fmt == "col_named":
                self._send(200, {"outputs": {"scores": scores}})
            else:
                self._send(200, {"outputs": scores})

    return Handler


class FMServer:
    """HTTP server + batcher around a loaded export (``start()`` runs it on a thread)."""

    def __init__(self, export_path: str, *, host: str = "127.0.0.1", port: int = 8501, model_name: str = "fm",
                 device: str | None = None, max_batch: int = 65536, batch_timeout_ms: float = 2.0):
        self.model = ServingModel.load(export_path, device)
        self.batcher = DynamicBatcher(self.model, max_batch, batch_timeout_ms)
        self.httpd = ThreadingHTTPServer((host, port), make_handler(self.batcher, model_name, self.model.meta))
        self.port = self.httpd.server_address[1]
        self._th: threading.Thread | None = None

    def start(self) -> "FMServer":
        self._th = threading.Thread(target=self.httpd.serve_forever, name="fm-http", daemon=True)
        self._th.start()
        return self

    def serve_forever(self) -> None:
        self.httpd.serve_forever()

    def close(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
        self.batcher.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Serve a fast_tffm_amd export over HTTP (TF-Serving REST API)")
    ap.add_argument("--dir", required=True, help="export directory written by run.py generate")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8501)
    ap.add_argument("--model-name", default="fm")
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-batch", type=int, default=65536, help="lines per coalesced model call")
    ap.add_argument("--batch-timeout-ms", type=float, default=2.0)
    a = ap.parse_args(argv)
    srv = FMServer(a.dir, host=a.host, port=a.port, model_name=a.model_name, device=a.device,
                   max_batch=a.max_batch, batch_timeout_ms=a.batch_timeout_ms)
    print(f"serving {a.dir} as '{a.model_name}' on http://{a.host}:{srv.port}/v1/models/{a.model_name}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    finally:
        srv.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
