"""HBM-resident training data: binary CSR caches uploaded once, batches gathered on the device.

MI355X has 288 GB of HBM; a 125M-row k=64 fp32 table shard with its Adagrad slots takes
~65 GB, so a pre-parsed dataset of tens of GB fits beside it.  ``DeviceDataset`` uploads
the ``.fmb`` caches (data/bincache.py) in file order; the native loader in rows mode
draws examples exactly like the text / binary paths (shuffle window, file order, rank
sharding, resume) and ships only their global row numbers + the batch's CSR offsets;
``hip/batch_gather.hip`` assembles the batch in HBM.  File-fed training then runs at
the device step rate instead of the host's copy or parse rate.
"""

from __future__ import annotations

import struct

import numpy as np
import torch

from ..ops import native

_HDR = struct.Struct("<8sIIqqqi20x")
MAGIC = b"FMCSR\x00v1"
F_VALS, F_WEIGHTS, F_HASHED = 1, 2, 4


def _align8(x: int) -> int:
    return (x + 7) & ~7


def read_header(path: str) -> dict:
    with open(path, "rb") as f:
        magic, ver, flags, n, nnz, vocab, mf = _HDR.unpack(f.read(_HDR.size))
    if magic != MAGIC or ver != 1:
        raise ValueError(f"{path}: not a version-1 binary CSR (.fmb) file")
    lab = _HDR.size
    p = _align8(lab + 4 * n)
    wts = p if flags & F_WEIGHTS else -1
    if flags & F_WEIGHTS:
        p = _align8(p + 4 * n)
    offs, ids = p, p + 8 * (n + 1)
    vals = _align8(ids + 4 * nnz) if flags & F_VALS else -1
    return dict(flags=flags, n=n, nnz=nnz, vocab_size=vocab, max_feats=mf, labels=lab, weights=wts, offsets=offs,
                ids=ids, vals=vals)


def dataset_bytes(files: list[str]) -> int:
    """Device bytes ``DeviceDataset`` needs for ``files``."""
    hs = [read_header(f) for f in files]
    any_vals = any(h["flags"] & F_VALS for h in hs)
    any_w = any(h["flags"] & F_WEIGHTS for h in hs)
    n, nnz = sum(h["n"] for h in hs), sum(h["nnz"] for h in hs)
    return n * (4 + 8 + (4 if any_w else 0)) + 8 + nnz * (4 + (4 if any_vals else 0))


class DeviceDataset:
    """The concatenation of ``files`` (in order) on ``device``: labels [N], weights [N] | None,
    offsets int64 [N + 1], ids int32 [nnz], vals [nnz] | None."""

    CHUNK = 64 << 20  # bytes per host -> device copy (the file is memory-mapped, never loaded whole)

    def __init__(self, files: list[str], device, vocab_size: int, hash_feature_id: bool = False):
        self.device = torch.device(device)
        hs = [read_header(f) for f in files]
        for f, h in zip(files, hs):
            if h["vocab_size"] != vocab_size or bool(h["flags"] & F_HASHED) != bool(hash_feature_id):
                raise ValueError(f"{f}: converted with vocabulary_size {h['vocab_size']}, hash_feature_id "
                                 f"{bool(h['flags'] & F_HASHED)}; the model uses {vocab_size}, {bool(hash_feature_id)}")
        ws = {bool(h["flags"] & F_WEIGHTS) for h in hs}
        if len(ws) > 1:
            raise ValueError("binary CSR caches disagree on weights")
        self.N = sum(h["n"] for h in hs)
        self.nnz = sum(h["nnz"] for h in hs)
        any_vals = any(h["flags"] & F_VALS for h in hs)
        dev = self.device
        self.labels = torch.empty(self.N, dtype=torch.float32, device=dev)
        self.weights = torch.empty(self.N, dtype=torch.float32, device=dev) if ws == {True} else None
        self.offsets = torch.empty(self.N + 1, dtype=torch.int64, device=dev)
        self.ids = torch.empty(self.nnz, dtype=torch.int32, device=dev)
        self.vals = torch.empty(self.nnz, dtype=torch.float32, device=dev) if any_vals else None
        self.offsets[:1].zero_()
        r = e = 0
        for f, h in zip(files, hs):
            mm = np.memmap(f, dtype=np.uint8, mode="r")

            def put(dst, off, count, dt, shift=0):
                isz = np.dtype(dt).itemsize
                step = max(1, self.CHUNK // isz)
                for i in range(0, count, step):
                    k = min(step, count - i)
                    a = np.frombuffer(mm, dtype=dt, count=k, offset=off + i * isz)
                    t = torch.from_numpy(a.copy() if shift == 0 else a + shift)
                    dst[i: i + k].copy_(t, non_blocking=False)

            n, z = h["n"], h["nnz"]
            put(self.labels[r: r + n], h["labels"], n, np.float32)
            if self.weights is not None:
                put(self.weights[r: r + n], h["weights"], n, np.float32)
            put(self.offsets[r + 1: r + n + 1], h["offsets"] + 8, n, np.int64, shift=e)
            put(self.ids[e: e + z], h["ids"], z, np.int32)
            if self.vals is not None:
                if h["vals"] >= 0:
                    put(self.vals[e: e + z], h["vals"], z, np.float32)
                else:
                    self.vals[e: e + z].fill_(1.0)
            r, e = r + n, e + z
            del mm
        if self.nnz:  # ids index the table: one check at load, none per batch
            lo, hi = int(self.ids.min()), int(self.ids.max())
            if lo < 0 or hi >= vocab_size:
                raise ValueError(f"binary CSR caches hold feature ids outside [0, {vocab_size})")

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.labels, self.weights, self.offsets, self.ids, self.vals)
                   if t is not None)

    def gather(self, rows: torch.Tensor, offsets: torch.Tensor, nnz: int, has_vals: bool, stream=None):
        """Assemble the batch of device ``rows`` (int64 [B]) with CSR ``offsets`` (int32 [B + 1],
        device) on ``stream``: returns (labels, ids, vals | None, weights | None)."""
        from ..ops.kernels import _p

        B = rows.numel()
        dev = self.device
        st = stream or torch.cuda.current_stream(dev)
        labels = torch.empty(B, dtype=torch.float32, device=dev)
        ids = torch.empty(nnz, dtype=torch.int32, device=dev)
        vals = torch.empty(nnz, dtype=torch.float32, device=dev) if has_vals and self.vals is not None else None
        weights = torch.empty(B, dtype=torch.float32, device=dev) if self.weights is not None else None
        if rows.dtype != torch.int64 or offsets.dtype != torch.int32 or offsets.numel() != B + 1:
            raise ValueError("rows must be int64 [B] and offsets int32 [B + 1]")
        native.hip().batch_gather(rows=_p(rows), boff=_p(offsets), B=B, N=self.N, src_off=_p(self.offsets),
                                  src_ids=_p(self.ids), src_vals=_p(self.vals), src_labels=_p(self.labels),
                                  src_weights=_p(self.weights), ids=_p(ids), vals=_p(vals), labels=_p(labels),
                                  weights=_p(weights), stream=st.cuda_stream)
        return labels, ids, vals, weights
