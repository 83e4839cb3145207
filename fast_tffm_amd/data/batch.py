"""A parsed mini-batch in CSR form.

The reference's input pipeline enqueues the 6-tuple
``(labels, weights, local_ids, ori_ids, vals, poses)`` (tffm/fm_model.py:75-78)
with ``tf.unique`` already applied.  Here the batch carries the raw global
feature ids; de-duplication runs on the device as part of the step
(ops.kernels.dedup), so the host side of the pipeline only parses.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class Batch:
    labels: torch.Tensor            # [B] float32
    offsets: torch.Tensor           # [B+1] int32 CSR row offsets (the reference's feature_poses)
    ids: torch.Tensor               # [nnz] int64 global feature ids in [0, vocabulary_size)
    vals: torch.Tensor | None       # [nnz] float32, None => all ones
    weights: torch.Tensor | None = None  # [B] float32, None => all ones
    nnz: int = -1                   # host copy of offsets[-1] (avoids a device sync)
    reader_pos: tuple | None = None  # (epoch, batches consumed in epoch) after this batch
    max_feats: int = -1             # host-known max features per example (-1: unknown)
    offsets_host: torch.Tensor | None = None  # CPU copy of offsets (lets the executor split without a sync)

    def __post_init__(self):
        if self.nnz < 0:
            self.nnz = int(self.ids.numel())

    @property
    def B(self) -> int:
        return int(self.labels.numel())

    @property
    def device(self) -> torch.device:
        return self.ids.device

    def _host_offsets(self) -> torch.Tensor | None:
        return self.offsets_host if self.offsets_host is not None else (
            self.offsets if self.offsets.device.type == "cpu" else None)

    def host_offset(self, i: int) -> int:
        """offsets[i] as a host int (a device read only when no host copy is known)."""
        h = self._host_offsets()
        return int(h[i]) if h is not None else int(self.offsets[i].item())

    def to(self, device, non_blocking: bool = True) -> "Batch":
        def mv(t):
            return None if t is None else t.to(device, non_blocking=non_blocking)

        return Batch(mv(self.labels), mv(self.offsets), mv(self.ids), mv(self.vals), mv(self.weights), self.nnz,
                     self.reader_pos, self.max_feats, self._host_offsets())

    def pin_memory(self) -> "Batch":
        def pn(t):
            return None if t is None else t.pin_memory()

        return Batch(pn(self.labels), pn(self.offsets), pn(self.ids), pn(self.vals), pn(self.weights), self.nnz,
                     self.reader_pos, self.max_feats, self._host_offsets())

    @staticmethod
    def from_parsed(labels: np.ndarray, sizes: np.ndarray, ids: np.ndarray, vals: np.ndarray,
                    weights: np.ndarray | None = None, drop_unit_vals: bool = True) -> "Batch":
        offsets = np.zeros(len(sizes) + 1, dtype=np.int32)
        np.cumsum(sizes, out=offsets[1:])
        v = torch.from_numpy(np.ascontiguousarray(vals, dtype=np.float32))
        if drop_unit_vals and v.numel() > 0 and bool((v == 1).all()):
            v = None  # all-ones values: the kernels take the x=1 fast path
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        if ids.size == 0 or int(ids.max()) < 2**31:
            ids = ids.astype(np.int32)  # table rows are int32 on the device
        return Batch(
            labels=torch.from_numpy(np.ascontiguousarray(labels, dtype=np.float32)),
            offsets=torch.from_numpy(offsets),
            ids=torch.from_numpy(ids),
            vals=v,
            weights=None if weights is None else torch.from_numpy(np.ascontiguousarray(weights, dtype=np.float32)),
            nnz=int(offsets[-1]),
            max_feats=int(sizes.max()) if len(sizes) else 0,
        )

    def slice(self, start: int, end: int) -> "Batch":
        """Examples [start, end) as a new batch (host tensors)."""
        o = self.offsets
        a, b = int(o[start]), int(o[end])
        return Batch(self.labels[start:end], (o[start:end + 1] - a).contiguous(), self.ids[a:b],
                     None if self.vals is None else self.vals[a:b],
                     None if self.weights is None else self.weights[start:end], b - a, max_feats=self.max_feats)
