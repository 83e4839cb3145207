"""Criteo-shaped synthetic batches, generated on the device.

Benchmarks cannot read Criteo-1TB (no network, and text parsing cannot feed
10^8 ex/s anyway: SURVEY.md §6.4), so the benchmark feeds batches with the
same *shape*: 39 features per example (13 integer fields bucketized to
categorical + 26 categorical fields), value 1, per-field power-law (Zipf)
value popularity with Criteo-1TB-like field cardinalities, hashed into the
global slot space with a 64-bit mixer (the moral equivalent of
``hash_feature_id = True``).  Labels are Bernoulli(0.25), like Criteo's CTR.
"""

from __future__ import annotations

import torch

from .batch import Batch

# Criteo-1TB categorical cardinalities (the 26 C-fields, as used by MLPerf DLRM),
# plus 13 integer fields bucketized to ~64 log-buckets each.
CRITEO_CAT_CARD = [
    39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546, 403346, 10, 2208, 11938, 155, 4,
    976, 14, 39979771, 25641295, 39664984, 585935, 12972, 108, 36,
]
CRITEO_INT_BUCKETS = [64] * 13
CRITEO_FIELD_CARD = CRITEO_INT_BUCKETS + CRITEO_CAT_CARD  # 39 fields


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic)."""
    x = x + (0x9E3779B97F4A7C15 - (1 << 64))
    x = (x ^ ((x >> 30) & ((1 << 34) - 1))) * (0xBF58476D1CE4E5B9 - (1 << 64))
    x = (x ^ ((x >> 27) & ((1 << 37) - 1))) * (0x94D049BB133111EB - (1 << 64))
    return x ^ ((x >> 31) & ((1 << 33) - 1))


def zipf_sample(n: int, card: int, alpha: float, gen: torch.Generator, device) -> torch.Tensor:
    """Approximate Zipf(alpha) over [0, card) by inverting the continuous power-law CDF."""
    u = torch.rand(n, generator=gen, device=device, dtype=torch.float64)
    if card <= 1:
        return torch.zeros(n, dtype=torch.int64, device=device)
    a = 1.0 - alpha
    # x in [1, card+1): F^-1(u) = ((card+1)^a - 1) u + 1)^(1/a)
    hi = float(card + 1) ** a
    x = ((hi - 1.0) * u + 1.0) ** (1.0 / a)
    return (x.floor().to(torch.int64) - 1).clamp_(0, card - 1)


class CriteoSynth:
    """Generator of Criteo-shaped CSR batches on ``device``."""

    def __init__(self, vocab_size: int, *, fields: list[int] | None = None, alpha: float = 1.1, seed: int = 1234,
                 device: torch.device | str = "cpu", ctr: float = 0.25):
        self.vocab_size = int(vocab_size)
        self.fields = list(fields or CRITEO_FIELD_CARD)
        self.F = len(self.fields)
        self.alpha = alpha
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.ctr = ctr

    def batch(self, B: int) -> Batch:
        dev = self.device
        cols = []
        for f, card in enumerate(self.fields):
            val = zipf_sample(B, card, self.alpha, self.gen, dev)
            h = _mix64(val * 64 + f)
            cols.append(torch.remainder(h, self.vocab_size))
        ids = torch.stack(cols, dim=1).reshape(-1)
        ids = (ids.to(torch.int32) if self.vocab_size < 2**31 else ids).contiguous()
        offsets = torch.arange(0, (B + 1) * self.F, self.F, dtype=torch.int32, device=dev)
        labels = (torch.rand(B, generator=self.gen, device=dev) < self.ctr).to(torch.float32)
        return Batch(labels=labels, offsets=offsets, ids=ids, vals=None, weights=None, nnz=B * self.F,
                     max_feats=self.F, offsets_host=torch.arange(0, (B + 1) * self.F, self.F, dtype=torch.int32))


def random_batch(B: int, vocab_size: int, max_feats: int = 8, *, seed: int = 0, device="cpu",
                 with_vals: bool = True, with_weights: bool = True, label_kind: str = "binary",
                 min_feats: int = 1) -> Batch:
    """Small random ragged CSR batch (tests): variable nnz per example, duplicates allowed."""
    g = torch.Generator().manual_seed(seed)
    sizes = torch.randint(min_feats, max_feats + 1, (B,), generator=g, dtype=torch.int32)
    offsets = torch.zeros(B + 1, dtype=torch.int32)
    offsets[1:] = torch.cumsum(sizes, 0)
    nnz = int(offsets[-1])
    ids = torch.randint(0, vocab_size, (nnz,), generator=g, dtype=torch.int64)
    vals = (torch.rand(nnz, generator=g) * 2 - 0.5) if with_vals else None
    if label_kind == "binary":
        labels = (torch.rand(B, generator=g) < 0.3).float()
    else:
        labels = torch.randn(B, generator=g)
    weights = (torch.rand(B, generator=g) + 0.5) if with_weights else None
    return Batch(labels, offsets, ids, vals, weights, nnz, max_feats=int(sizes.max()) if B else 0).to(device)


def write_libsvm(path: str, n_lines: int, *, shape: str = "criteo", vocab_size: int = 1_000_000, seed: int = 0,
                 weights_path: str | None = None, with_values: bool = False) -> None:
    """Write a synthetic libsvm text file in the reference's input format
    (``<label> <fid>[:<val>] ...``, README.md:44-50).

    shape="criteo": 39 fields (13 bucketized integer + 26 categorical, Zipf
    popularity), 16-39 features per line like the reference's sample data
    (SURVEY.md §6.3); shape="a1a": LIBSVM a1a-shaped (123 binary features,
    ~14 active per line).  ``weights_path`` gets one weight per line (2 for
    label 1, 1 for label 0, like the reference's data/weight_*).
    """
    import numpy as np

    rng = np.random.default_rng(seed)
    lines, wl = [], []
    if shape == "a1a":
        base = rng.random(123) ** 3
        for _ in range(n_lines):
            k = int(rng.integers(11, 15))
            feats = np.sort(rng.choice(123, size=k, replace=False, p=base / base.sum()))
            label = int(rng.random() < 0.24 + 0.5 * (feats[0] < 10))
            toks = [f"{int(f) + 1}:1" if with_values else str(int(f) + 1) for f in feats]
            lines.append(f"{label} " + " ".join(toks))
            wl.append("2" if label else "1")
    else:
        cards = CRITEO_FIELD_CARD
        for _ in range(n_lines):
            nf = int(rng.integers(16, 40))
            fields = np.sort(rng.choice(39, size=nf, replace=False))
            toks = []
            for f in fields:
                card = cards[f]
                val = min(int(rng.zipf(1.3)) - 1, card - 1)
                fid = (f * 1_000_003 + val * 7919) % vocab_size
                toks.append(f"{fid}:{rng.random():.3f}" if with_values else str(fid))
            label = int(rng.random() < 0.25)
            lines.append(f"{label} " + " ".join(toks))
            wl.append("2" if label else "1")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    if weights_path:
        with open(weights_path, "w") as f:
            f.write("\n".join(wl) + "\n")
