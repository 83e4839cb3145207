"""Parameter table of the FM: hashed feature id -> (w, v[0..K)).

Reference: ``vocabulary_block_num`` TF variables ``vocab_block_i`` of shape
``[vocabulary_size // N + 1, K + 1]``, global id ``g`` in block ``g % N`` row
``g // N``, column 0 = w, columns 1..K = v (tffm/fm_model.py:269-291), plus the
Adagrad slot per variable.

Here one process owns one *shard* of rows with the same "mod" rule over the
data-parallel world (``owner = g % world``, ``local row = g // world``).  The
storage is HBM-friendly rather than reference-shaped:

* ``v``   [rows, Kp]  fp32, bf16 or fp8 (OCP e4m3, GPU only), Kp = K padded to
  whole lanes (pads are 0);
* ``w``   [rows]      fp32 (linear weight, kept separate so v rows stay aligned);
  fp8 tables store [w, scale, |v|^2, pad] rows (``wx`` [rows, 4], ``w`` = wx[:, 0]) so the
  row's dequantisation scale (a power of two) and squared norm arrive with w;
* ``s0v``/``s0w``     optimizer slot 0 (Adagrad accumulator / FTRL n);
* ``s1v``/``s1w``     optimizer slot 1 (FTRL z);
  fp32, except ``s0v`` / ``s1v`` of fp8 tables: bf16 with stochastic rounding
  (``K.state_dtype``), half the state bytes next to factors of 3 mantissa bits.

The checkpoint module converts to and from the reference layout.
"""

from __future__ import annotations

import math

import torch

from ..ops import kernels as K
from ..ops import native


def rows_per_shard(vocab_size: int, world: int) -> int:
    return (vocab_size + world - 1) // world


def shard_rows(vocab_size: int, world: int, rank: int) -> int:
    """Rows owned by ``rank``: ids g with g % world == rank and g < vocab_size."""
    return max(0, (vocab_size - rank + world - 1) // world)


class FMTable:
    def __init__(self, vocab_size: int, factor_num: int, *, world: int = 1, rank: int = 0,
                 dtype: torch.dtype = torch.float32, opt: K.OptConfig | None = None, init_range: float = 0.01,
                 seed: int = 0, device: torch.device | str = "cpu", init: bool = True, rows_multiple: int = 1):
        self.vocab_size = int(vocab_size)
        self.K = int(factor_num)
        self.world, self.rank = int(world), int(rank)
        self.dtype = dtype
        self.Kp = K.padded_k(self.K, dtype)
        self.opt = opt or K.OptConfig()
        self.device = torch.device(device)
        # allocated rows: the shard's ids, rounded up to ``rows_multiple`` (the replicated table of
        # the dense data-parallel step is cut into equal row slices, one per rank: dead rows at the
        # end are zero and never addressed)
        m = max(1, int(rows_multiple))
        self.real_rows = shard_rows(self.vocab_size, self.world, self.rank)
        self.rows = max(1, -(-self.real_rows // m) * m)
        self.init_range = float(init_range)
        self.seed = int(seed)
        dev = self.device
        self.fp8 = dtype == K.FP8
        if self.fp8 and self.device.type != "cuda":
            raise ValueError("fp8 tables run on the GPU kernels only")
        self.v = torch.zeros((self.rows, self.Kp), dtype=dtype, device=dev)
        if self.fp8:
            # [w, scale, |v|^2, pad] per row: the kernels read the scale at w[row * 4 + 1] and the
            # squared norm of the dequantised row (hip/fm_common.h fp8_norm2) at w[row * 4 + 2]
            self.wx = torch.zeros((self.rows, 4), dtype=torch.float32, device=dev)
            self.wx[:, 1] = 1.0
            self.w = self.wx[:, 0]
            self.scale = self.wx[:, 1]
            self.norm2 = self.wx[:, 2]
        else:
            self.wx = None
            self.w = torch.zeros(self.rows, dtype=torch.float32, device=dev)
            self.scale = self.norm2 = None
        acc0 = float(self.opt.initial_accumulator)
        n_state = max(1, self.opt.n_state)  # kernels always address slot 0
        sdt = self.state_dtype = K.state_dtype(dtype)
        self.s0v = torch.full((self.rows, self.Kp), acc0 if self.opt.name in ("adagrad", "ftrl") else 0.0,
                              dtype=sdt, device=dev)
        self.s0w = torch.full((self.rows,), acc0 if self.opt.name in ("adagrad", "ftrl") else 0.0,
                              dtype=torch.float32, device=dev)
        self.s1v = torch.zeros((self.rows, self.Kp), dtype=sdt, device=dev) if n_state > 1 else None
        self.s1w = torch.zeros((self.rows,), dtype=torch.float32, device=dev) if n_state > 1 else None
        if init:
            self.reinit()

    # ------------------------------------------------------------------
    @property
    def saved_rows(self) -> int:
        """Rows a checkpoint / reference view covers: the allocated rows without the dead padding
        of ``rows_multiple`` (an empty shard keeps its one allocated row)."""
        return max(1, min(self.rows, self.real_rows))

    @property
    def state(self) -> K.TableState:
        return K.TableState(self.v, self.w, self.s0v, self.s1v, self.s0w, self.s1w)

    def reinit(self, seed: int | None = None) -> None:
        """U(-r, r) over w and v[:K] as a pure function of (seed, global id, column)."""
        seed = self.seed if seed is None else int(seed)
        args = dict(v=self.v.data_ptr(), v_stride=self.v.stride(0), w=self.w.data_ptr(), w_stride=self.w.stride(0),
                    rows=self.rows, K=self.K, Kp=self.Kp, dtype=K.dtype_code(self.dtype), gid_mul=self.world,
                    gid_add=self.rank, seed=seed & 0xFFFFFFFFFFFFFFFF, range=self.init_range)
        if self.device.type == "cuda":
            native.hip().init_rows(**args, stream=torch.cuda.current_stream(self.device).cuda_stream)
        else:
            native.cpu().init_rows(**args)
        self._zero_dead_rows()

    def _zero_dead_rows(self) -> None:
        # the last shard may own fewer real ids than allocated rows (rows >= 1, rows_multiple)
        real = self.real_rows
        if real < self.rows:
            self.v[real:].zero_()
            self.w[real:].zero_()
            if self.scale is not None:
                self.scale[real:] = 1.0
                self.norm2[real:] = 0.0

    def adopt_fp8_rows(self, local_rows: torch.Tensor | None = None) -> None:
        """After fp8 rows and scales were written as stored bytes (checkpoint restore): rows whose
        scale is not a power of two (written before scales were; the scaled conversion in the
        forward applies only a scale's exponent) are re-quantised from their dequantised values,
        then the rows' norms are recomputed.  ``local_rows``: only these rows were written (an index
        tensor), else all."""
        if not self.fp8:
            return
        rows = None if local_rows is None else _as_index(local_rows, self.device)
        mant, _ = torch.frexp(self.scale if rows is None else self.scale[rows])
        bad = torch.nonzero(mant != 0.5).flatten()
        if rows is not None:
            bad = rows[bad]
        if bad.numel():
            self.set_v(bad, self.dense_v(bad)[:, : self.K])  # (refreshes the norms of these rows)
        self.refresh_norms(rows)

    def refresh_norms(self, local_rows: torch.Tensor | None = None) -> None:
        """Recompute the fp8 rows' |v|^2 column from the stored rows and scales (after writing v or
        the scales from the host side; the kernels keep it current themselves) -- of every row, or
        of ``local_rows`` (an index tensor) only."""
        if not self.fp8:
            return
        h = native.hip()
        st = torch.cuda.current_stream(self.device).cuda_stream
        kw = dict(v=self.v.data_ptr(), v_stride=self.v.stride(0), w=self.wx.data_ptr(), w_stride=self.wx.stride(0),
                  Kp=self.Kp, stream=st)
        if local_rows is None:
            h.fp8_row_norms(rows=self.rows, **kw)
            return
        idx = _as_index(local_rows, self.device)
        if idx.numel():
            h.fp8_row_norms(rows=idx.numel(), idx=idx.data_ptr(), **kw)

    def global_ids(self) -> torch.Tensor:
        return torch.arange(self.rows, device=self.device, dtype=torch.int64) * self.world + self.rank

    def nbytes(self) -> int:
        tot = 0
        for t in (self.v, self.wx if self.fp8 else self.w, self.s0v, self.s0w, self.s1v, self.s1w):
            if t is not None:
                tot += t.numel() * t.element_size()
        return tot

    # ------------------------------------------------------------------
    def reference_rows(self, local_rows: torch.Tensor | None = None) -> torch.Tensor:
        """Rows in the reference layout [n, K+1] (col 0 = w, cols 1..K = v), fp32."""
        if local_rows is None:
            n = self.saved_rows
            v, w = self.dense_v(slice(0, n)), self.w[:n]
        else:
            v, w = self.dense_v(local_rows), self.w[local_rows]
        return torch.cat([w.unsqueeze(1), v[:, : self.K].float()], dim=1)

    def dense_v(self, local_rows: torch.Tensor | None = None) -> torch.Tensor:
        """v rows as fp32 values (fp8: dequantised with the row scales)."""
        v = self.v if local_rows is None else self.v[local_rows]
        if not self.fp8:
            return v
        s = self.scale if local_rows is None else self.scale[local_rows]
        return v.float() * s[:, None]

    def set_v(self, local_rows: torch.Tensor | None, vals: torch.Tensor) -> None:
        """Write fp32 values into v[:, :K] (fp8: re-quantised per row, pads stay 0)."""
        if self.fp8:
            n = vals.shape[0]
            full = torch.zeros((n, self.Kp), dtype=torch.float32, device=self.device)
            full[:, : self.K] = vals.to(self.device, torch.float32)
            q, s = K.quantize_fp8_rows(full)
            if local_rows is None:
                self.v[:n], self.scale[:n] = q, s
                self.refresh_norms(torch.arange(n, device=self.device))
            else:
                self.v[local_rows], self.scale[local_rows] = q, s
                self.refresh_norms(local_rows)
            return
        vals = vals.to(self.device, self.dtype)
        if local_rows is None:
            self.v[: vals.shape[0], : self.K] = vals
        else:
            self.v[local_rows, : self.K] = vals

    def load_reference_rows(self, local_rows: torch.Tensor, rows_ref: torch.Tensor,
                            acc_ref: torch.Tensor | None = None) -> None:
        """Write reference-layout rows ([n, K+1]) and optional Adagrad slot rows into this shard."""
        rows_ref = rows_ref.to(self.device, torch.float32)
        self.w[local_rows] = rows_ref[:, 0]
        self.set_v(local_rows, rows_ref[:, 1:])
        if acc_ref is not None:
            acc_ref = acc_ref.to(self.device, torch.float32)
            self.s0w[local_rows] = acc_ref[:, 0]
            self.s0v[local_rows, : self.K] = acc_ref[:, 1:]

    def memory_report(self) -> str:
        gb = self.nbytes() / 2**30
        return (f"table shard rank {self.rank}/{self.world}: {self.rows} rows x K={self.K} (Kp={self.Kp}, "
                f"{str(self.dtype).replace('torch.', '')}), opt={self.opt.name}: {gb:.2f} GiB")


def _as_index(rows, device) -> torch.Tensor:
    """Row selection (index tensor or slice) -> contiguous int64 indices on ``device``."""
    if isinstance(rows, slice):
        return torch.arange(rows.start or 0, rows.stop, device=device, dtype=torch.int64)
    return rows.to(device=device, dtype=torch.int64).contiguous().flatten()


def bits_for(n: int) -> int:
    """Number of key bits needed to represent values in [0, n)."""
    return max(1, int(math.ceil(math.log2(max(n, 2)))))
