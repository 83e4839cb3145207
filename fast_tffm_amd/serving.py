"""Serving export (``run.py generate``) and a standalone predictor.

Reference: ``generate`` restores the latest checkpoint and writes a TF
SavedModel (tag ``serve``, signature ``serving_default``, input ``data_lines``
(string), output ``scores``, method PREDICT; run_tffm.py:93-120) whose graph is
pure TF: ``serving_parser`` splits feature-only lines ``id:val id:val ...``
(``:val`` mandatory, no label column), ``serving_scorer`` looks the ids up in
``vocab_block_i`` with the "mod" partition and evaluates the FM densely
(tffm/fm_model.py:195-265).  The export path must not exist yet.

Here the export directory holds both forms::

    export_path/saved_model.pb                      TF SavedModel of the reference's serving graph
    export_path/variables/variables.{index,data-*}  its variables (TF V2 tensor bundle)
    export_path/saved_model.json                    signature + model metadata (native predictor)
    export_path/variables/vocab_block_{i}.npy       reference layout [V // N + 1, K + 1]

(utils/saved_model.py writes the SavedModel without TensorFlow; its parity with TF's loader
is unpinned, checked by an independent numpy interpreter of the graph in the tests.)

``ServingModel.load(export_path).predict(data_lines)`` reproduces the
signature (lines -> scores) with the native scorer (CPU or gfx950), and
``python -m fast_tffm_amd.serving --dir export_path --inputs data.npy`` mirrors
``saved_model_cli run ... --inputs data_lines=data.npy``.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

SIGNATURE = {
    "tag_set": "serve",
    "signature_def": "serving_default",
    "method_name": "tensorflow/serving/predict",
    "inputs": {"data_lines": {"dtype": "string", "shape": [-1]}},
    "outputs": {"scores": {"dtype": "float32", "shape": [-1]}},
}


def export_model(ckpt_dir: str, export_path: str, *, vocabulary_block_num: int, hash_feature_id: bool = False,
                 loss_type: str = "mse") -> str:
    """Write a serving export of checkpoint ``ckpt_dir`` to the (new) directory ``export_path``."""
    from .utils.checkpoint import export_reference_blocks, read_meta

    if os.path.exists(export_path):
        raise FileExistsError(f"export path {export_path} already exists (it must not be a pre-existing directory)")
    meta = read_meta(ckpt_dir)
    tmp = export_path.rstrip("/") + ".tmp-export"
    os.makedirs(os.path.join(tmp, "variables"), exist_ok=True)
    export_reference_blocks(ckpt_dir, os.path.join(tmp, "variables"), vocabulary_block_num, with_slots=False)
    doc = dict(SIGNATURE)
    doc.update({
        "format": "fast_tffm_amd/serving-v1",
        "vocabulary_size": meta["vocabulary_size"],
        "vocabulary_block_num": vocabulary_block_num,
        "factor_num": meta["factor_num"],
        "hash_feature_id": bool(hash_feature_id),
        "loss_type": loss_type,
        "global_step": meta["global_step"],
        "global_bias": meta.get("global_bias"),
        "score": "raw FM score (logit for logistic loss)" + (" incl. the global bias" if meta.get("global_bias")
                                                             is not None else ", no global bias"),
    })
    with open(os.path.join(tmp, "saved_model.json"), "w") as f:
        json.dump(doc, f, indent=1)
    from .utils.saved_model import write_saved_model

    blocks = [np.load(os.path.join(tmp, "variables", f"vocab_block_{i}.npy"), mmap_mode="r", allow_pickle=False)
              for i in range(vocabulary_block_num)]
    write_saved_model(tmp, blocks, meta["vocabulary_size"], meta["factor_num"], global_bias=meta.get("global_bias"))
    del blocks
    os.replace(tmp, export_path)
    return export_path


def parse_serving_lines(lines, vocab_size: int, hash_feature_id: bool = False, threads: int = 4):
    """Feature-only lines ``id:val id:val ...`` -> (offsets, ids, vals) (reference serving_parser,
    tffm/fm_model.py:195-220: whitespace-split tokens, ``:val`` mandatory, no label column).

    Tokens are normalised to single spaces and parsed by the native multi-threaded parser
    behind a dummy label; a line whose ':' count differs from its token count has a token
    without a value (or with two) and is rejected like the reference's reshape([-1, 2])."""
    from .ops import native

    norm = []
    for ln in lines:
        if isinstance(ln, str):
            ln = ln.encode()
        toks = ln.split()
        if ln.count(b":") != len(toks):
            bad = next((t for t in toks if t.count(b":") != 1), b"")
            raise ValueError(f"serving input needs id:val tokens, got {bad.decode(errors='replace')!r}")
        norm.append(b"0 " + b" ".join(toks))
    _, sizes, ids, vals = native.cpu().parse_lines(norm, int(vocab_size), bool(hash_feature_id), int(threads))
    offsets = np.zeros(len(sizes) + 1, dtype=np.int32)
    np.cumsum(sizes, out=offsets[1:])
    return torch.from_numpy(offsets), torch.from_numpy(ids), torch.from_numpy(vals)


class ServingModel:
    """Loaded serving export: ``predict(data_lines) -> scores``."""

    def __init__(self, meta: dict, v: torch.Tensor, w: torch.Tensor, device: torch.device):
        self.meta, self.v, self.w, self.device = meta, v, w, device
        self.K = meta["factor_num"]
        self.Kp = v.shape[1]

    @classmethod
    def load(cls, export_path: str, device: str | None = None) -> "ServingModel":
        from .ops.kernels import padded_k

        with open(os.path.join(export_path, "saved_model.json")) as f:
            meta = json.load(f)
        V, K, N = meta["vocabulary_size"], meta["factor_num"], meta["vocabulary_block_num"]
        dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        Kp = padded_k(K)
        v = torch.zeros((V, Kp), dtype=torch.float32)
        w = torch.zeros(V, dtype=torch.float32)
        gid = torch.arange(V)
        for i in range(N):
            blk = np.load(os.path.join(export_path, "variables", f"vocab_block_{i}.npy"), mmap_mode="r",
                          allow_pickle=False)
            sel = gid[gid % N == i]
            rows = torch.from_numpy(np.ascontiguousarray(blk[(sel // N).numpy()]))
            w[sel] = rows[:, 0]
            v[sel, :K] = rows[:, 1:]
        return cls(meta, v.to(dev), w.to(dev), dev)

    def _parse_gpu(self, flat: list):
        """GPU tokenizer (hip/parse.hip) over the lines behind a dummy label, ':value' required;
        None when a line is outside its syntax subset (then the CPU path decides / raises)."""
        from .ops import kernels as Kn

        enc = [ln.encode() if isinstance(ln, str) else bytes(ln) for ln in flat]
        data = b"".join(b"0 " + ln + b"\n" for ln in enc)
        starts = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum([len(ln) + 3 for ln in enc], out=starts[1:])
        d = self.device
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(d, non_blocking=False)
        pg = Kn.parse_gpu(buf, torch.from_numpy(starts).to(d), self.meta["vocabulary_size"],
                          self.meta["hash_feature_id"], require_vals=True)
        if pg.fallback:
            return None
        vals = pg.vals if pg.vals is not None else torch.ones(pg.nnz, dtype=torch.float32, device=d)
        return pg.offsets, pg.ids, vals

    def predict(self, data_lines) -> np.ndarray:
        from .ops import kernels as Kn

        flat = np.asarray(data_lines).reshape(-1).tolist()
        d = self.device
        parsed = self._parse_gpu(flat) if d.type == "cuda" and flat else None
        if parsed is None:
            offsets, ids, vals = parse_serving_lines(flat, self.meta["vocabulary_size"],
                                                     self.meta["hash_feature_id"])
        else:
            offsets, ids, vals = parsed
        gb = self.meta.get("global_bias")
        bias = torch.tensor([gb], dtype=torch.float32, device=d) if gb is not None else None
        fo = Kn.fm_forward(offsets.to(d), ids.to(torch.int32).to(d), vals.to(d), self.v, self.w, self.Kp,
                           want_r1=False, bias=bias)
        return fo.pred.cpu().numpy()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Run a fast_tffm_amd serving export (saved_model_cli run equivalent)")
    ap.add_argument("--dir", required=True)
    ap.add_argument("--inputs", required=True, help="data_lines=FILE.npy | FILE.npy | FILE.txt (one line each)")
    ap.add_argument("--outdir", default=None)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    path = a.inputs.split("=", 1)[1] if "=" in a.inputs else a.inputs
    if path.endswith(".npy"):
        lines = np.load(path, allow_pickle=False)
    else:
        with open(path) as f:
            lines = [ln.rstrip("\n") for ln in f]
    m = ServingModel.load(a.dir, a.device)
    scores = m.predict(lines)
    if a.outdir:
        os.makedirs(a.outdir, exist_ok=True)
        np.save(os.path.join(a.outdir, "scores.npy"), scores)
    print("Result for output key scores:")
    print(scores)
    return 0


if __name__ == "__main__":
    sys.exit(main())
