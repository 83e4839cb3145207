"""Typed, validated wrappers over the native step kernels.

Every wrapper dispatches on the device of its tensors: CUDA (HIP) tensors go to
the gfx950 kernels of ``_fm_hip``, CPU tensors to ``_fm_cpu``.  Launches are
asynchronous on the current torch stream; nothing here synchronises the host
unless ``FM_DEBUG_CHECKS=1`` asks for index range checks.

Row layout contract (see csrc/hip/fm_common.h): a factor table ``v`` is
``[rows, Kp]`` (fp32 or bf16, Kp padded so that a lane moves 16 bytes), the
linear weights ``w`` are a separate fp32 vector (or column ``Kp`` of a packed
``[rows, Kp+4]`` exchange buffer, passed as a strided view).
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import native

LOSS_TYPES = {"none": 0, "mse": 1, "logistic": 2}
OPT_TYPES = {"adagrad": 0, "ftrl": 1, "sgd": 2}
BWD_LOCAL, BWD_EMIT = 0, 1
BWD_EMIT_TABLE = 2   # params from table rows uniq[u]; gradient scattered to grad_out[uniq[u]] + touch mark

_DEBUG = os.environ.get("FM_DEBUG_CHECKS", "0") == "1"


def debug_checks() -> bool:
    """FM_DEBUG_CHECKS=1: index range checks in the kernel wrappers and exchange split checks."""
    return _DEBUG


def set_debug_checks(on: bool) -> None:
    global _DEBUG
    _DEBUG = bool(on)


def set_fwd_mfma(on: bool) -> bool:
    """Route fp8 k=128 binary-feature forwards to the matrix-core kernel (hip/fm_fwd_mfma.hip: the "mfma"
    build variant only, where it is the default; the default module has no such kernel and stays on the
    VALU kernel) or the VALU kernel; returns the previous setting."""
    h = native.hip()
    was = bool(h.fwd_mfma_enabled())
    h.set_fwd_mfma(bool(on))
    return was


FP8 = torch.float8_e4m3fn   # OCP e4m3 table storage (+ fp32 scale per row), GPU only
FP8_MAX = 448.0


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return 0
    if t == torch.bfloat16:
        return 1
    if t == FP8:
        return 2
    raise TypeError(f"unsupported table dtype {t}; use float32, bfloat16 or float8_e4m3fn")


def elems_per_lane(dtype: torch.dtype) -> int:
    """Table elements one lane moves per row access: 4 (16 B fp32, 8 B bf16, 4 B fp8)."""
    return 4


def padded_k(K: int, dtype: torch.dtype = torch.float32) -> int:
    """Factor columns stored per row: K rounded up to whole lanes (multiples of 4)."""
    e = elems_per_lane(dtype)
    return ((K + e - 1) // e) * e


def r1_dtype(table_dtype: torch.dtype) -> torch.dtype:
    """Storage dtype of the forward's r1 cache [B, Kp] for a table dtype: fp32, or bf16 for fp8
    tables (3-bit factor mantissas; bf16 r1 halves the backward's per-occurrence gather --
    hip/fm_common.h R1Bf16)."""
    return torch.bfloat16 if table_dtype == FP8 else torch.float32


def fp8_row_scale(m: torch.Tensor) -> torch.Tensor:
    """Row scales of fp8 rows with largest |value| m (hip/fm_common.h fp8_row_scale): the power of
    two s with m / s in (224, 448]; 1 for empty rows."""
    m = m.float()
    t = torch.clamp(m / FP8_MAX, min=2.0 ** -126)
    mant, e = torch.frexp(t)  # t = mant * 2^e, mant in [0.5, 1)
    s = torch.where(mant == 0.5, t, torch.ldexp(torch.ones_like(t), e))
    return torch.where(m > 0, s, torch.ones_like(m))


def quantize_fp8_rows(vals: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row fp8 quantisation (the kernels' store_row): scale = fp8_row_scale(max|v|) (a power of
    two), q = rne(v / scale)."""
    v = vals.float()
    m = v.abs().amax(dim=1) if v.shape[1] else torch.zeros(v.shape[0], device=v.device)
    s = fp8_row_scale(m)
    q = (v * (1.0 / s)[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, s


@dataclass
class OptConfig:
    name: str = "adagrad"
    lr: float = 0.01
    l1: float = 0.0
    l2: float = 0.0
    beta: float = 0.0
    initial_accumulator: float = 0.1

    @property
    def code(self) -> int:
        return OPT_TYPES[self.name]

    @property
    def n_state(self) -> int:
        return 2 if self.name == "ftrl" else (1 if self.name == "adagrad" else 0)


def _p(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t: torch.Tensor) -> int:
    """The current HIP stream's handle on ``t``'s device (the raw accessor: the Stream-object path costs
    several Python calls per kernel launch, ~16 launches per sharded step)."""
    idx = t.device.index
    if _raw_stream is not None and idx is not None:
        return _raw_stream(idx)
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _chk_vec(t: torch.Tensor | None, dtype: torch.dtype, n: int | None, name: str, dev: torch.device) -> None:
    if t is None:
        return
    _check(t.dtype == dtype, f"{name}: expected {dtype}, got {t.dtype}")
    _check(t.device == dev, f"{name}: expected device {dev}, got {t.device}")
    _check(t.is_contiguous(), f"{name}: must be contiguous")
    if n is not None:
        _check(t.numel() >= n, f"{name}: needs >= {n} elements, has {t.numel()}")


def _chk_rows(v: torch.Tensor, Kp: int, name: str) -> int:
    """Validate a row-major factor source and return its row stride in elements."""
    _check(v.dim() == 2, f"{name}: expected 2-D rows")
    _check(v.stride(1) == 1, f"{name}: rows must be contiguous")
    epl = elems_per_lane(v.dtype)
    _check(Kp % epl == 0, f"{name}: Kp={Kp} must be a multiple of {epl} for {v.dtype}")
    _check(v.shape[1] >= Kp, f"{name}: has {v.shape[1]} columns < Kp={Kp}")
    _check(v.stride(0) % epl == 0, f"{name}: row stride {v.stride(0)} must be a multiple of {epl}")
    _check(v.data_ptr() % 16 == 0, f"{name}: base must be 16-byte aligned")
    return v.stride(0)


def _range_check(idx: torch.Tensor, hi: int, name: str) -> None:
    if _DEBUG and idx.numel() > 0 and not (idx.is_cuda and torch.cuda.is_current_stream_capturing()):
        lo_v, hi_v = int(idx.min()), int(idx.max())
        _check(lo_v >= 0 and hi_v < hi, f"{name}: index range [{lo_v}, {hi_v}] outside [0, {hi})")


# ---------------------------------------------------------------------------
# forward
# ---------------------------------------------------------------------------
class FwdOut:
    """Outputs of fm_forward. ``loss_sum``/``regv``/``regw`` are 0-d tensors on the op's device."""

    __slots__ = ("pred", "r1", "dpred", "loss_sum", "regv", "regw", "loss_partial")

    def __init__(self, pred, r1, dpred, loss_sum, regv, regw, loss_partial=None):
        self.pred, self.r1, self.dpred = pred, r1, dpred
        self.loss_sum, self.regv, self.regw = loss_sum, regv, regw
        self.loss_partial = loss_partial  # per-workgroup loss sums when the reduction was deferred

    def finish_loss(self) -> torch.Tensor | None:
        """The summed loss; a deferred reduction (``fm_forward(defer_loss=True)``) is enqueued now,
        on the current stream."""
        if self.loss_sum is None and self.loss_partial is not None:
            self.loss_sum = self.loss_partial.sum(dtype=torch.float32)
        return self.loss_sum


def fm_forward(offsets: torch.Tensor, rows: torch.Tensor, vals: torch.Tensor | None, v: torch.Tensor,
               w: torch.Tensor, Kp: int, *, labels: torch.Tensor | None = None,
               weights: torch.Tensor | None = None, loss: str = "none", grad_scale: float = 1.0,
               want_r1: bool = True, want_reg: bool = False, pred: torch.Tensor | None = None,
               r1: torch.Tensor | None = None, dpred: torch.Tensor | None = None,
               partial: torch.Tensor | None = None, threads: int = 0,
               bias: torch.Tensor | None = None, self_rows: SelfRows | None = None,
               seg_lookup: "SegIndex | None" = None, defer_loss: bool = False, max_feats: int = -1) -> FwdOut:
    """FM score of a CSR batch (reference FmScorer, cc/fm_scorer_op.h:101-140), fused with the loss.

    pred_i = sum_j x_j w_j + 1/2 sum_k [(sum_j x_j v_jk)^2 - sum_j x_j^2 v_jk^2]  (+ bias[0], optional
    global bias; the reference has none, fm_scorer_op.h:134-136)
    With ``loss`` in {mse, logistic} also returns the summed weighted loss and
    ``dpred = grad_scale * dL_i/dpred_i``.

    ``self_rows`` (GPU, ``rows`` = segment ids): segments in its range read this rank's table.
    ``seg_lookup`` (GPU): ``rows`` are the dedup's keys and every occurrence's segment (its
    row of ``v``) is found through the bucket index (``seg_index``) instead of an inverse map.
    (``defer_loss``, GPU: the per-workgroup loss partials are left for ``FwdOut.finish_loss``, so the
    reduction can be enqueued after the backward instead of between forward and backward.)
    ``max_feats`` (host-known maximum occurrences per example, -1 unknown): lets fp8 k=128 batches of
    binary features run on the matrix cores (hip/fm_fwd_mfma.hip).
    """
    dev = rows.device
    B = offsets.numel() - 1
    _chk_vec(offsets, torch.int32, B + 1, "offsets", dev)
    nnz = rows.numel()
    _chk_vec(rows, torch.int32, nnz, "rows", dev)
    _chk_vec(vals, torch.float32, nnz, "vals", dev)
    v_stride = _chk_rows(v, Kp, "v")
    _check(w.dim() == 1 or (w.dim() == 2 and w.shape[1] == 1), "w: expected a vector (possibly strided)")
    _check(w.dtype == torch.float32 and w.device == dev, "w: expected float32 on the rows' device")
    w_stride = w.stride(0)
    _check(w.shape[0] >= v.shape[0], "w: fewer rows than v")
    # fp8 rows: w is the row tails [w, scale, |v|^2, .] (Table rows / wire rows): the forward reads all three
    _check(v.dtype != FP8 or w_stride >= 3, "fp8 rows: w must be a strided view of [w, scale, |v|^2, .] row tails")
    lt = LOSS_TYPES[loss]
    if bias is not None:
        _chk_vec(bias, torch.float32, 1, "bias", dev)
    if lt:
        _chk_vec(labels, torch.float32, B, "labels", dev)
        _chk_vec(weights, torch.float32, B, "weights", dev)
    if seg_lookup is None:
        _range_check(rows, v.shape[0], "rows")
    else:
        _check(_is_gpu(rows), "segment lookup is a GPU path")
    if pred is None:
        pred = torch.empty(B, dtype=torch.float32, device=dev)
    if want_r1 and r1 is None:
        r1 = torch.empty((B, Kp), dtype=r1_dtype(v.dtype), device=dev)
    if want_r1:
        _check(r1.dtype == r1_dtype(v.dtype) and r1.is_contiguous() and r1.shape[1] == Kp and r1.shape[0] >= B,
               f"r1: contiguous [B, Kp] {r1_dtype(v.dtype)} for a {v.dtype} table")
    if not want_r1:
        r1 = None
    if lt and dpred is None:
        dpred = torch.empty(B, dtype=torch.float32, device=dev)
    dt = dtype_code(v.dtype)
    host_checks = _DEBUG and not (offsets.is_cuda and torch.cuda.is_current_stream_capturing())
    if host_checks and max_feats is not None and max_feats >= 0 and B > 0:
        _check(int((offsets[1:] - offsets[:-1]).max()) <= max_feats, "max_feats: an example has more features")
    if host_checks and v.dtype == FP8 and w_stride == 4 and v.shape[0] > 0:
        # table rows [w, scale, |v|^2, .]: the kernels apply only the scale's exponent, so every host
        # write of v / scale must keep scales powers of two (FMTable.set_v / adopt_fp8_rows do)
        sc = torch.as_strided(w, (v.shape[0],), (4,), w.storage_offset() + 1)
        _check(bool((torch.frexp(sc)[0] == 0.5).all()), "fp8 table: a row scale is not a power of two")
    if _is_gpu(rows):
        h = native.hip()
        grid = h.fwd_grid(max(B, 1))
        if partial is None or partial.numel() < 3 * grid:
            partial = torch.zeros(3 * grid, dtype=torch.float32, device=dev)
        lp = partial[:grid]
        rp = partial[grid:3 * grid]
        dkw = {}
        if self_rows is not None and self_rows.u1 > self_rows.u0:
            _self_check(self_rows, v, None)
            dkw["self_rows"] = self_rows.packed()
        h.fwd(B=B, offsets=_p(offsets), rows=_p(rows), vals=_p(vals), v=_p(v), v_stride=v_stride, w=_p(w),
              w_stride=w_stride, Kp=Kp, dtype=dt, labels=_p(labels), weights=_p(weights), loss_type=lt,
              grad_scale=float(grad_scale), pred=_p(pred), r1=_p(r1), dpred=_p(dpred) if lt else 0,
              loss_partial=_p(lp) if lt else 0, reg_partial=_p(rp) if want_reg else 0, grid=grid,
              stream=_stream(rows), bias=_p(bias),
              seg_idx=_p(seg_lookup.idx) if seg_lookup is not None else 0,
              seg_keys=_p(seg_lookup.keys) if seg_lookup is not None else 0,
              seg_shift=seg_lookup.shift if seg_lookup is not None else 0,
              max_feats=int(max_feats) if max_feats is not None else -1, **dkw)
        # (an in-kernel last-block reduction was measured slower: the per-block agent-scope
        # release fence writes back L2 -- fwd 211 -> 412 us; a separate reduce is ~10 us; the same
        # reduce on a second stream beside the backward measured slower too: 0.668-0.671 -> 0.676 ms,
        # profiles/r3/loss_stream_ab.txt)
        # A sum by the chunk backward's first workgroup (no reduce kernel between forward and
        # backward) made the chunk kernel itself ~30% slower even when not taken -- a workgroup
        # barrier in the chunk kernel changes its code (k64 0.668 -> 0.88 ms, same box;
        # profiles/r3/fused_loss_ab.txt)
        # (the local step defers this reduction past the backward: nothing reads the loss before it)
        loss_sum = lp.sum(dtype=torch.float32) if lt and not defer_loss else None
        regv = rp.view(grid, 2)[:, 0].sum() if want_reg else None
        regw = rp.view(grid, 2)[:, 1].sum() if want_reg else None
        if lt and defer_loss:
            return FwdOut(pred, r1, dpred, None, regv, regw, loss_partial=lp)
    else:
        _check(self_rows is None, "self rows are a GPU path")
        c = native.cpu()
        ls, rv, rw = c.fwd(B=B, offsets=_p(offsets), rows=_p(rows), vals=_p(vals), v=_p(v), v_stride=v_stride,
                           w=_p(w), w_stride=w_stride, Kp=Kp, dtype=dt, labels=_p(labels), weights=_p(weights),
                           loss_type=lt, grad_scale=float(grad_scale), pred=_p(pred), r1=_p(r1),
                           dpred=_p(dpred) if lt else 0, threads=threads, bias=_p(bias))
        loss_sum = torch.tensor(ls, dtype=torch.float32) if lt else None
        regv = torch.tensor(rv, dtype=torch.float32) if want_reg else None
        regw = torch.tensor(rw, dtype=torch.float32) if want_reg else None
    return FwdOut(pred, r1, dpred if lt else None, loss_sum, regv, regw)


# ---------------------------------------------------------------------------
# dedup
# ---------------------------------------------------------------------------
class DedupOut:
    """Grouping of a batch's occurrences by key (sorted unique keys = segments).

    ``counts`` is a 2-element int32 device tensor (U, #chunks) -- no host sync;
    ``num_unique`` is a view of counts[0]; ``U_host`` is set on CPU and after
    ``.sync()``.  ``perm`` is the sorted payload: the occurrence index, unless
    the dedup ran with the example index as payload (then ``sorted_ex is perm``).
    """

    __slots__ = ("n", "skeys", "perm", "uniq", "seg_start", "seg_chunk", "chunk_start", "chunk_seg", "chunk_key",
                 "counts", "num_unique", "inv", "sorted_ex", "sorted_x", "U_host", "CH", "big_list", "big_count",
                 "multi", "ex_shift", "bwd_fresh")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw.get(k))

    def sync(self) -> int:
        if self.U_host is None:
            # counts[7]: the in-tree sort's look-back verdict (nonzero: this grouping is invalid)
            u, err = self.counts[0:8:7].tolist() if self.counts.numel() >= 8 else (int(self.num_unique.item()), 0)
            if err:
                raise RuntimeError(f"dedup: the radix sort's look-back spin bound was hit (error word {err}); "
                                   "this batch's grouping is invalid")
            self.U_host = int(u)
        return self.U_host

    def unique_keys(self) -> torch.Tensor:
        return self.uniq[: self.sync()]


class DedupWorkspace:
    """Reusable device buffers for dedup + chunk plan of up to ``cap`` occurrences."""

    def __init__(self, cap: int, device: torch.device, CH: int = 32):
        self.cap, self.device, self.CH = cap, device, CH
        n1 = max(cap, 1)
        i32 = dict(dtype=torch.int32, device=device)
        self.iota = torch.arange(n1, **i32)
        self.skeys = torch.empty(n1, **i32)
        self.perm = torch.empty(n1, **i32)
        self.uniq = torch.empty(n1, **i32)
        self.seg_start = torch.empty(n1 + 1, **i32)
        self.seg_chunk = torch.empty(n1 + 1, **i32)
        self.chunk_start = torch.empty(n1 + 1, **i32)
        self.chunk_seg = torch.empty(n1, **i32)   # segment id | first (bit 30) | single (bit 31)
        self.chunk_key = torch.empty(n1, **i32)
        self.counts = torch.zeros(8, **i32)   # U, #chunks, #multi-chunk rows, -, bwd big rows, -
        self.multi = torch.empty(n1, **i32)
        self.inv = torch.empty(n1, **i32)
        self.sorted_ex = torch.empty(n1, **i32)
        self.sorted_x = torch.empty(n1, dtype=torch.float32, device=device)
        self.ex_of_occ = torch.empty(n1, **i32)
        self.big_list = torch.empty(n1, **i32)
        self.big_count = self.counts[4:5]     # zeroed with the counts by every GPU dedup
        if device.type == "cuda":
            nbytes = native.hip().dedup_workspace_bytes(n1)
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        else:
            self.ws = None


DEV_ERR_SORT = 1  # hip/fm_common.h kDevErrSort


def check_device_errors(device: torch.device | None = None, clear: bool = True) -> None:
    """Raise if a kernel on ``device`` (default: the current GPU) flagged an invalid result in the
    module's sticky error word since the last check (synchronises the device).  Kernels that cannot
    fail loudly without a host sync set it -- the in-tree radix sort when a look-back spin bound is
    hit -- and the bench / trainer check it at their reporting points.  No-op without a GPU."""
    if device is not None and device.type != "cuda":
        return
    if not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
        err = int(native.hip().device_errors(clear))
    if err:
        what = ["radix sort look-back spin bound hit (a dedup plan was invalid)"] if err & DEV_ERR_SORT else []
        raise RuntimeError(f"device error word {err:#x}: {'; '.join(what) or 'unknown'}")


_SORT_CHECKED: set = set()


def _sort_selfcheck(dev: torch.device) -> None:
    """Once per device and process, before the in-tree sort first groups a batch: its passes are
    stable only if the LDS returns ds_add_rtn ranks in ascending lane order for lanes of one
    instruction that hit the same counter (radix_sort.hip rs_rank_wave) -- measured on gfx950, not
    documented.  Sort a digit-colliding pattern against torch's stable sort; on a mismatch switch the
    dedup to rocPRIM's sort (bitwise the same order) and warn."""
    if dev.index in _SORT_CHECKED or torch.cuda.is_current_stream_capturing():
        return
    _SORT_CHECKED.add(dev.index)
    h = native.hip()
    if not h.sort_algo():
        return
    g = torch.Generator(device="cpu").manual_seed(7)
    n = 3 * 8192 + 77  # several tiles, a partial last one
    keys = (torch.randint(0, 6, (n,), generator=g) * 0x01010101 + torch.randint(0, 2, (n,), generator=g)).to(
        torch.int32).to(dev)  # every digit of every pass collides heavily
    vals = torch.arange(n, dtype=torch.int32, device=dev)
    ko, vo = radix_sort(keys, vals, key_bits=32)
    ref_k, ref_v = torch.sort(keys.long(), stable=True)
    if not (torch.equal(ko.long(), ref_k) and torch.equal(vo, ref_v.to(torch.int32))):
        import warnings

        h.set_sort_algo(0)
        warnings.warn("in-tree radix sort failed its stability self-check on this device: the dedup uses "
                      "rocPRIM's sort (FM_SORT=rocprim)")


def set_sort_algo(algo: str) -> str:
    """The dedup's sort backend: "fm" (in-tree onesweep radix sort, hip/radix_sort.hip, default) or
    "rocprim" (rocPRIM's onesweep; same stable order); returns the previous one.  FM_SORT=rocprim at
    start-up too."""
    _check(algo in ("rocprim", "fm"), f"sort backend {algo!r}: rocprim or fm")
    h = native.hip()
    was = "fm" if h.sort_algo() else "rocprim"
    h.set_sort_algo(1 if algo == "fm" else 0)
    return was


def radix_sort(keys: torch.Tensor, vals: torch.Tensor, key_bits: int = 32) -> tuple[torch.Tensor, torch.Tensor]:
    """Stable sort of int32 (key, value) pairs by the keys' low ``key_bits`` bits on the in-tree
    radix sort (GPU): returns (sorted keys, values in the same order)."""
    n = keys.numel()
    _chk_vec(keys, torch.int32, n, "keys", keys.device)
    _chk_vec(vals, torch.int32, n, "vals", keys.device)
    _check(_is_gpu(keys), "radix_sort is a GPU kernel")
    h = native.hip()
    ko, vo = torch.empty_like(keys), torch.empty_like(vals)
    ws = torch.empty(max(1, int(h.radix_sort_ws_bytes(n))), dtype=torch.uint8, device=keys.device)
    h.radix_sort(keys=_p(keys), vals=_p(vals), kout=_p(ko), vout=_p(vo), n=n, end_bit=int(key_bits), ws=_p(ws),
                 ws_bytes=ws.numel(), stream=_stream(keys))
    return ko, vo


def slot_bits_for(B: int, max_feats: int) -> int:
    """Bits of the in-example slot of a packed occurrence code, or 0 when codes do not fit int32."""
    if max_feats is None or max_feats < 1:
        return 0
    sb = max(1, (max_feats - 1).bit_length())
    return sb if (B << sb) < 2**31 else 0


def csr_rows(offsets: torch.Tensor, out: torch.Tensor | None = None, nnz: int | None = None,
             slot_bits: int = 0) -> torch.Tensor:
    """Example index of every CSR occurrence (the reference gets it implicitly from feature_poses).

    With ``slot_bits > 0`` (GPU) the packed code ``example << slot_bits | slot`` instead:
    the dedup sort carries it and decodes example and occurrence index from it.
    """
    B = offsets.numel() - 1
    if nnz is None:
        nnz = int(offsets[-1])
    if out is None:
        out = torch.empty(nnz, dtype=torch.int32, device=offsets.device)
    if _is_gpu(offsets):
        native.hip().csr_rows(B=B, offsets=_p(offsets), ex_of_occ=_p(out), slot_bits=int(slot_bits),
                              stream=_stream(offsets))
    else:
        _check(slot_bits == 0, "packed occurrence codes are a GPU path")
        native.cpu().csr_rows(B=B, offsets=_p(offsets), ex_of_occ=_p(out))
    return out


# FM_DEDUP_FUSE=0: the dedup's producers (shard_keys, csr_rows) as separate kernels (A/B switch)
_FUSE_PRODUCERS = os.environ.get("FM_DEDUP_FUSE", "1") != "0"


def dedup(keys: torch.Tensor, *, ws: DedupWorkspace | None = None, key_bits: int = 32,
          ex_of_occ: torch.Tensor | None = None, vals: torch.Tensor | None = None, want_inv: bool = False,
          CH: int | None = None, want_perm: bool = False, num_examples: int | None = None,
          Kp: int | None = None, ex_shift: int = 0, offsets: torch.Tensor | None = None,
          gen_codes: bool = False, shard_ids: torch.Tensor | None = None,
          shard: tuple[int, int] | None = None) -> DedupOut:
    """Sort-based unique over non-negative int32 keys (reference tf.unique, fm_model.py:72).

    Unique keys come out in ascending order (the reference's first-occurrence
    order is an implementation detail no result depends on).  On the GPU the
    result also carries the backward's chunk plan.  When neither the inverse
    map, per-occurrence values nor the occurrence permutation are needed, the
    sort carries the example index directly (one gather pass less).
    (``num_examples`` / ``Kp`` are accepted for interface stability; the plan does not use them.)

    Fused producers (GPU; folded into the in-tree sort's histogram / first pass, the separate kernels
    first under FM_SORT=rocprim): ``gen_codes`` -- the occurrence codes ``csr_rows(offsets,
    slot_bits=ex_shift)`` (``ex_of_occ`` not given); ``shard_ids`` + ``shard = (world, rows_per_shard)``
    -- ``keys`` is the OUTPUT buffer of ``shard_keys(shard_ids, ...)``.
    """
    dev = keys.device
    n = keys.numel()
    _chk_vec(keys, torch.int32, n, "keys", dev)
    if ws is None or ws.cap < n:
        ws = DedupWorkspace(max(n, 1), dev, CH or 32)
    CH = CH or ws.CH
    fuse_ids = 0
    if shard_ids is not None:
        _check(shard is not None and shard_ids.numel() == n, "shard_ids needs shard=(world, rows_per_shard)")
        if _FUSE_PRODUCERS and _is_gpu(keys) and shard_ids.dtype == torch.int32 and shard_ids.is_contiguous():
            _check(shard[0] * shard[1] < 2**31, "sharded keys must fit int32")
            fuse_ids = _p(shard_ids)
        else:
            shard_keys(shard_ids, shard[0], shard[1], keys)
    fuse_codes = False
    if gen_codes:
        _check(ex_of_occ is None and offsets is not None, "gen_codes: offsets, no ex_of_occ")
        in_payload = _is_gpu(keys) and not want_perm and (ex_shift > 0 or (vals is None and not want_inv))
        ex_of_occ = ws.ex_of_occ[:n]
        if _FUSE_PRODUCERS and in_payload and offsets.numel() > 1:
            fuse_codes = True     # written into ex_of_occ only by the rocPRIM backend's csr_rows
        else:
            csr_rows(offsets, out=ex_of_occ, nnz=n, slot_bits=ex_shift)
    if ex_of_occ is not None:
        _chk_vec(ex_of_occ, torch.int32, n, "ex_of_occ", dev)
    if vals is not None:
        _chk_vec(vals, torch.float32, n, "vals", dev)
    key_bits = max(1, min(32, int(key_bits)))
    packed = ex_shift > 0
    if packed:  # ex_of_occ holds packed codes (csr_rows slot_bits): the payload decodes to example + occurrence
        _check(_is_gpu(keys) and ex_of_occ is not None and offsets is not None and not want_perm,
               "packed occurrence codes need the GPU, codes and offsets")
    ex_payload = ex_of_occ is not None and _is_gpu(keys) and not want_perm and (
        packed or (vals is None and not want_inv))
    out = DedupOut(n=n, skeys=ws.skeys, perm=ws.perm, uniq=ws.uniq, seg_start=ws.seg_start,
                   seg_chunk=ws.seg_chunk, chunk_start=ws.chunk_start, chunk_seg=ws.chunk_seg,
                   chunk_key=ws.chunk_key, counts=ws.counts,
                   num_unique=ws.counts[:1], inv=ws.inv if want_inv else None,
                   sorted_ex=(ws.perm if ex_payload else ws.sorted_ex) if ex_of_occ is not None else None,
                   sorted_x=ws.sorted_x if vals is not None else None, CH=CH, big_list=ws.big_list,
                   big_count=ws.big_count, multi=ws.multi, ex_shift=int(ex_shift))
    if _is_gpu(keys):
        h = native.hip()
        _check(1 <= CH <= h.MAX_CH, f"CH must be in [1, {h.MAX_CH}]")
        _sort_selfcheck(dev)
        h.dedup(n=n, end_bit=key_bits, CH=CH, keys=_p(keys), payload=_p(ex_of_occ if ex_payload else ws.iota),
                skeys=_p(ws.skeys), spay=_p(ws.perm), uniq=_p(ws.uniq), seg_start=_p(ws.seg_start),
                seg_chunk=_p(ws.seg_chunk), chunk_start=_p(ws.chunk_start), chunk_seg=_p(ws.chunk_seg),
                chunk_key=_p(ws.chunk_key),
                counts=_p(ws.counts), inv=_p(out.inv),
                ex_of_occ=0 if ex_payload else _p(ex_of_occ),
                sorted_ex=0 if ex_payload else _p(out.sorted_ex), vals=_p(vals), sorted_x=_p(out.sorted_x),
                payload_is_ex=int(ex_payload), ex_shift=int(ex_shift), offsets=_p(offsets),
                ws=_p(ws.ws), ws_bytes=ws.ws.numel(), stream=_stream(keys), ids=fuse_ids,
                kW=int(shard[0]) if fuse_ids else 1, kRps=int(shard[1]) if fuse_ids else 0,
                gen_codes=int(fuse_codes), B=offsets.numel() - 1 if fuse_codes else 0)
        out.bwd_fresh = True  # the backward counters were zeroed on this stream
    else:
        U = native.cpu().dedup(n=n, keys=_p(keys), skeys=_p(ws.skeys), perm=_p(ws.perm), uniq=_p(ws.uniq),
                               seg_start=_p(ws.seg_start), inv=_p(out.inv), ex_of_occ=_p(ex_of_occ),
                               sorted_ex=_p(out.sorted_ex), vals=_p(vals), sorted_x=_p(out.sorted_x))
        ws.counts[0] = U
        out.U_host = U
    return out


# ---------------------------------------------------------------------------
# backward (+ optimizer)
# ---------------------------------------------------------------------------
@dataclass
class TableState:
    """Parameters and optimizer slots of one (local) table shard."""

    v: torch.Tensor                 # [rows, Kp] fp32 / bf16 / fp8
    w: torch.Tensor                 # [rows] fp32
    s0v: torch.Tensor | None = None  # adagrad accumulator / ftrl n   [rows, Kp] state_dtype(v.dtype)
    s1v: torch.Tensor | None = None  # ftrl z                          [rows, Kp] state_dtype(v.dtype)
    s0w: torch.Tensor | None = None  # [rows] fp32
    s1w: torch.Tensor | None = None  # [rows] fp32

    def __post_init__(self):
        want = state_dtype(self.v.dtype)
        for name in ("s0v", "s1v"):
            t = getattr(self, name)
            _check(t is None or t.dtype == want, f"{name}: {want} optimizer state for a {self.v.dtype} table")


def state_dtype(table_dtype: torch.dtype) -> torch.dtype:
    """Storage of the per-factor optimizer state: fp32, bf16 for fp8 tables (hip/fm_common.h
    StateBf16: 8 mantissa bits with stochastic rounding next to factors carrying 3; halves the
    state bytes of the row read-modify-write)."""
    return torch.bfloat16 if table_dtype == FP8 else torch.float32


@dataclass
class SelfRows:
    """Row-sharded step (GPU): segments ``[u0, u1)`` of a batch's sorted unique keys ``keys``
    are this rank's own table rows (row = key - ``base``).  ``fm_forward`` / ``fm_backward``
    read them from ``table`` instead of the gathered wire rows, and the backward applies the
    optimizer in place to the exclusive ones (``excl`` int32 [u1 - u0], 1 = no other rank
    requested the row this step; None = all, world 1) -- hip/fm_common.h SelfRows."""

    u0: int
    u1: int
    base: int
    keys: torch.Tensor
    table: TableState
    excl: torch.Tensor | None = None

    def packed(self) -> list[int]:
        """The binding's form: [u0, u1, base, keys, excl, v, v_stride, w, w_stride]."""
        t = self.table
        return [self.u0, self.u1, self.base, _p(self.keys), _p(self.excl), _p(t.v), t.v.stride(0), _p(t.w),
                t.w.stride(0)]


def _self_check(sr: SelfRows, v: torch.Tensor, keys: torch.Tensor | None) -> None:
    _check(sr.table.v.dtype == v.dtype, "self rows: the table and the wire rows must share the dtype")
    _check(keys is None or sr.keys.data_ptr() == keys.data_ptr(), "self rows: keys must be the dedup's uniq")
    _check(0 <= sr.u0 <= sr.u1, "self rows: bad segment range")
    if sr.excl is not None:
        _chk_vec(sr.excl, torch.int32, None, "self excl", v.device)
        _check(sr.excl.numel() >= sr.u1 - sr.u0, "self excl too short")


@dataclass
class SegIndex:
    """Bucket index over a dedup's sorted unique keys (``seg_index``): key -> segment."""

    idx: torch.Tensor     # int32 [nb + 1]
    keys: torch.Tensor    # the dedup's uniq (sorted keys)
    shift: int


def seg_lookup_enabled() -> bool:
    """Row-sharded step: segment lookup through a bucket index instead of the dedup's inverse
    map (FM_SEG_LOOKUP, default on; profiles/r2/inv_cost.txt)."""
    return os.environ.get("FM_SEG_LOOKUP", "1") != "0"


def seg_index_bits(nnz: int, key_bits: int) -> tuple[int, int]:
    """(shift, nb) of the key-bucket index: nb ~ nnz / 4 buckets (a power of two in [16, 2^20],
    at most 2^key_bits), bucket = key >> shift over ``key_bits``-bit keys.  A Criteo-shaped
    batch (5.1M occurrences, ~378k unique keys) gets 2^20 buckets: ~0.4 keys per bucket."""
    bb = max(4, min(20, max(1, nnz).bit_length() - 2, key_bits))
    shift = max(0, key_bits - bb)
    return shift, 1 << (key_bits - shift)


def seg_index(dd: DedupOut, key_bits: int, out: torch.Tensor | None = None) -> SegIndex:
    """Build the bucket index of ``dd``'s unique keys on the current stream (GPU, no host sync)."""
    _check(_is_gpu(dd.uniq), "seg_index is a GPU path")
    shift, nb = seg_index_bits(dd.n, key_bits)
    if out is None or out.numel() < nb + 1:
        out = torch.empty(nb + 1, dtype=torch.int32, device=dd.uniq.device)
    native.hip().seg_index(n_max=int(dd.n), uniq=_p(dd.uniq), counts=_p(dd.counts), shift=int(shift), nb=int(nb),
                           idx=_p(out), stream=_stream(dd.uniq))
    return SegIndex(out, dd.uniq, shift)


def partial_rows(n: int, CH: int) -> int:
    """Upper bound on backward chunks (= partial rows) for n occurrences: U + n / CH."""
    return max(n, 1) + max(n, 1) // max(CH, 1) + 1


def fm_backward(dd: DedupOut, dpred: torch.Tensor, r1: torch.Tensor, Kp: int, *, mode: int,
                table: TableState | None = None, opt: OptConfig | None = None,
                src_v: torch.Tensor | None = None, src_w: torch.Tensor | None = None,
                grad_out: torch.Tensor | None = None, reg_v: float = 0.0, reg_w: float = 0.0,
                partial: torch.Tensor | None = None, threads: int = 0, grad_bf16: bool = False,
                sr_counter: torch.Tensor | None = None,
                seg_bounds: torch.Tensor | None = None, piece: int = -1,
                self_rows: SelfRows | None = None) -> torch.Tensor | None:
    """Segmented FM backward over the dedup grouping (reference FmGrad, cc/fm_grad_op.h:59-163).

    Per unique row u with occurrences (i, x):
      g_v = sum x*dpred_i*(r1_i - x*v) + reg_v * n_u * v
      g_w = sum x*dpred_i            + reg_w * n_u * w
    mode=BWD_LOCAL applies ``opt`` in place on ``table`` rows ``uniq[u]``;
    mode=BWD_EMIT writes [g_v, g_w] rows into ``grad_out[u]`` (``src_v``/``src_w``
    hold the gathered parameter rows in unique order).  ``piece`` 0 / 1 with
    ``seg_bounds`` (GPU, int32 [2W+1]) reduces only the segments of every owner's first /
    second part (split backward of the row-sharded exchange); piece 1 must follow piece 0.
    ``self_rows`` (GPU, EMIT): segments in its range are read from its table; the exclusive ones
    get ``opt`` applied in place (with ``sr_counter``) and no gradient row.
    """
    dev = dpred.device
    _check(dd.sorted_ex is not None, "dedup must be run with ex_of_occ")
    _chk_vec(dpred, torch.float32, None, "dpred", dev)
    _check(r1.is_contiguous() and r1.shape[1] == Kp, "r1: [B, Kp] contiguous")
    if mode == BWD_EMIT_TABLE:
        _check(_is_gpu(dpred) and table is not None and grad_out is not None,
               "EMIT_TABLE mode: GPU, table (parameter rows) + dense grad_out")
        v, w = table.v, table.w
        dt = dtype_code(v.dtype)
        s0v = s1v = s0w = s1w = None
        s_stride = 0
        _check(grad_out.dtype == torch.float32 and grad_out.stride(1) == 1 and grad_out.shape[0] >= v.shape[0],
               "grad_out: dense fp32 rows covering the table")
        gstride, gptr = grad_out.stride(0), grad_out.data_ptr()
        g_wcol = Kp
        _check(gstride >= Kp + 2 and gstride % 4 == 0, "grad_out rows: [g_v | g_w | touch | ...], stride % 4 == 0")
    elif mode == BWD_LOCAL:
        _check(table is not None and opt is not None, "LOCAL mode needs table + opt")
        v, w = table.v, table.w
        dt = dtype_code(v.dtype)
        _check(opt.name == "sgd" or table.s0v is not None, "optimizer state missing")
        s_stride = table.s0v.stride(0) if table.s0v is not None else 0
        s0v, s1v, s0w, s1w = table.s0v, table.s1v, table.s0w, table.s1w
        if opt.name == "sgd":  # kernels always touch s0: give them scratch
            s0v, s0w, s_stride = (table.s0v, table.s0w, s_stride)
        gstride, gptr = 0, 0
    else:
        _check(src_v is not None and src_w is not None and grad_out is not None, "EMIT mode needs src + grad_out")
        v, w = src_v, src_w
        dt = dtype_code(v.dtype)  # gathered wire rows: fp32, bf16 or fp8 (+ scale at w + 1)
        s0v = s1v = s0w = s1w = None
        s_stride = 0
        _check(grad_out.dtype == torch.float32 and grad_out.stride(1) == 1, "grad_out: fp32 rows")
        gstride, gptr = grad_out.stride(0), grad_out.data_ptr()
        g_wcol = (Kp * 2 + 15) // 16 * 4 if grad_bf16 else Kp
        _check(gstride >= g_wcol + 1 and gstride % 4 == 0,
               "grad_out row stride must hold the w column and be a multiple of 4")
        _check(not grad_bf16 or _is_gpu(dpred), "bf16 gradient rows are a GPU path")
        if self_rows is not None and self_rows.u1 > self_rows.u0:
            _check(_is_gpu(dpred) and opt is not None, "self rows: GPU path with the optimizer")
            _self_check(self_rows, v, dd.uniq)
            t = self_rows.table
            s0v, s1v, s0w, s1w = t.s0v, t.s1v, t.s0w, t.s1w
            _check(s0v is not None and s0w is not None, "self rows: the table's optimizer state")
            s_stride = s0v.stride(0)
    v_stride = _chk_rows(v, Kp, "v")
    _check(r1.dtype == r1_dtype(v.dtype), f"r1: {r1_dtype(v.dtype)} for {v.dtype} rows (the forward's r1)")
    o = opt or OptConfig()
    if piece >= 0:
        _check(_is_gpu(dpred) and seg_bounds is not None and mode in (BWD_EMIT, BWD_EMIT_TABLE),
               "split backward pieces: GPU, EMIT / EMIT_TABLE, seg_bounds")
        _chk_vec(seg_bounds, torch.int32, 3, "seg_bounds", dev)
    if _is_gpu(dpred):
        h = native.hip()
        if partial is None:
            partial = torch.empty((partial_rows(dd.n, dd.CH), Kp + 4), dtype=torch.float32, device=dev)
        _check(partial.numel() >= partial_rows(dd.n, dd.CH) * (Kp + 4), "partial scratch too small")
        skw = {}
        if mode == BWD_EMIT and self_rows is not None and self_rows.u1 > self_rows.u0:
            skw = dict(self_rows=self_rows.packed())
        h.bwd(mode=mode, counts=_p(dd.counts), chunk_start=_p(dd.chunk_start), chunk_seg=_p(dd.chunk_seg),
              chunk_key=_p(dd.chunk_key),
              seg_start=_p(dd.seg_start), seg_chunk=_p(dd.seg_chunk), uniq=_p(dd.uniq),
              sorted_ex=_p(dd.sorted_ex), ex_shift=int(dd.ex_shift or 0), sorted_x=_p(dd.sorted_x),
              dpred=_p(dpred), r1=_p(r1), Kp=Kp,
              v=_p(v), v_stride=v_stride, w=_p(w), w_stride=w.stride(0), s0v=_p(s0v), s1v=_p(s1v),
              s_stride=s_stride, s0w=_p(s0w), s1w=_p(s1w), reg_v=float(reg_v), reg_w=float(reg_w),
              opt_type=o.code, lr=float(o.lr), l1=float(o.l1), l2=float(o.l2), beta=float(o.beta),
              grad_out=gptr, g_stride=gstride, partial=_p(partial), big_list=_p(dd.big_list),
              big_count=_p(dd.big_count), multi=_p(dd.multi), nex=int(dpred.numel()), dtype=dt, max_chunks=dd.n,
              max_unique=dd.n,
              stream=_stream(dpred), g_wcol=g_wcol if mode != BWD_LOCAL else -1, g_bf16=int(bool(grad_bf16)),
              sr_counter=_p(sr_counter), counters_ready=int(bool(dd.bwd_fresh)),
              seg_bounds=_p(seg_bounds), piece=int(piece),
              n_owners=(seg_bounds.numel() - 1) // 2 if seg_bounds is not None else 0, **skw)
        dd.bwd_fresh = False  # a second backward over this grouping zeroes its counters itself
    else:
        _check(self_rows is None, "self rows are a GPU path")
        U = dd.sync()
        native.cpu().bwd(mode=mode, U=U, seg_start=_p(dd.seg_start), uniq=_p(dd.uniq), sorted_ex=_p(dd.sorted_ex),
                         sorted_x=_p(dd.sorted_x), dpred=_p(dpred), r1=_p(r1), Kp=Kp, v=_p(v), v_stride=v_stride,
                         w=_p(w), w_stride=w.stride(0), s0v=_p(s0v), s1v=_p(s1v), s_stride=s_stride, s0w=_p(s0w),
                         s1w=_p(s1w), reg_v=float(reg_v), reg_w=float(reg_w), opt_type=o.code, lr=float(o.lr),
                         l1=float(o.l1), l2=float(o.l2), beta=float(o.beta), grad_out=gptr, g_stride=gstride,
                         dtype=dt, threads=threads)
    return grad_out


# ---------------------------------------------------------------------------
# row-sharded helpers
# ---------------------------------------------------------------------------
def gather_rows(req: torch.Tensor, table: TableState, Kp: int, out: torch.Tensor, threads: int = 0,
                skip: tuple[int, int] | None = None) -> torch.Tensor:
    """out[p] = [v[req[p]], w[req[p]], 0...] (fp32), the owner side of a sharded lookup.
    ``skip`` (GPU): requests [s0, s1) are left out (their ``out`` rows are not written)."""
    dev = req.device
    R = req.numel()
    _chk_vec(req, torch.int32, R, "req", dev)
    v_stride = _chk_rows(table.v, Kp, "v")
    _check(out.dtype == torch.float32 and out.stride(1) == 1 and out.shape[0] >= R, "out: fp32 rows")
    _check(out.stride(0) >= Kp + 4 and out.stride(0) % 4 == 0, "out row stride")
    _range_check(req, table.v.shape[0], "req")
    dt = dtype_code(table.v.dtype)
    if _is_gpu(req):
        s0, s1 = skip or (0, 0)
        _check(0 <= s0 <= s1 <= R, "gather skip range")
        native.hip().gather_rows(R=R, req=_p(req), v=_p(table.v), v_stride=v_stride, w=_p(table.w),
                                 w_stride=table.w.stride(0), Kp=Kp, dtype=dt, out=_p(out), o_stride=out.stride(0),
                                 stream=_stream(req), skip0=s0, skip1=s1)
    else:
        _check(skip is None, "gather skip ranges are a GPU path")
        native.cpu().gather_rows(R=R, req=_p(req), v=_p(table.v), v_stride=v_stride, w=_p(table.w),
                                 w_stride=table.w.stride(0), Kp=Kp, dtype=dt, out=_p(out), o_stride=out.stride(0),
                                 threads=threads)
    return out


def shard_keys(ids: torch.Tensor, world: int, rows_per_shard: int, out: torch.Tensor) -> torch.Tensor:
    """Sharded key of every occurrence: (id % world) * rows_per_shard + id // world (int32)."""
    n = ids.numel()
    _check(world * rows_per_shard < 2**31, "sharded keys must fit int32")
    if _is_gpu(ids) and ids.dtype == torch.int32:
        _chk_vec(out, torch.int32, None, "out", ids.device)
        _check(out.numel() >= n, "out too small")
        native.hip().shard_keys(n=n, ids=_p(ids), W=int(world), Rps=int(rows_per_shard), keys=_p(out),
                                stream=_stream(ids))
        return out[:n]
    keys = (ids % world) * rows_per_shard + torch.div(ids, world, rounding_mode="floor")
    out[:n].copy_(keys)
    return out[:n]


def owner_counts(dd: DedupOut, rows_per_shard: int, world: int, out: torch.Tensor | None = None,
                 out2: torch.Tensor | None = None) -> torch.Tensor:
    """int64[world]: unique keys (owner * rows_per_shard + row) per owner, computed without a host sync.
    ``out`` / ``out2``: 1-D int64 views (any stride) to write (``out2``: a second copy, GPU)."""
    if out is None:
        out = torch.empty(world, dtype=torch.int64, device=dd.uniq.device)
    _check(out.dtype == torch.int64 and out.dim() == 1 and out.numel() == world, "owner_counts out: int64[world]")
    if dd.uniq.device.type == "cuda":
        if out2 is not None:
            _check(out2.dtype == torch.int64 and out2.shape == out.shape and out2.stride() == out.stride()
                   and out2.device == out.device, "owner_counts out2: like out")
        native.hip().owner_counts(uniq=_p(dd.uniq), num_unique=_p(dd.num_unique), Rps=int(rows_per_shard), W=world,
                                  out=_p(out), stream=_stream(dd.uniq), stride=out.stride(0),
                                  out2=_p(out2) if out2 is not None else 0)
    else:
        owner = torch.div(dd.uniq[: dd.sync()].to(torch.int64), rows_per_shard, rounding_mode="floor")
        out.copy_(torch.bincount(owner, minlength=world))
        if out2 is not None:
            out2.copy_(out)
    return out


def apply_rows(dd: DedupOut, grad_in: torch.Tensor, table: TableState, opt: OptConfig, Kp: int,
               threads: int = 0, sr_counter: torch.Tensor | None = None) -> None:
    """Owner side of a sharded update: sum received grad rows per table row, then one optimizer step."""
    v_stride = _chk_rows(table.v, Kp, "v")
    _check(grad_in.dtype == torch.float32 and grad_in.stride(1) == 1, "grad_in: fp32 rows")
    dt = dtype_code(table.v.dtype)
    s_stride = table.s0v.stride(0) if table.s0v is not None else 0
    if _is_gpu(grad_in):
        native.hip().apply_rows(num_unique=_p(dd.num_unique), seg_start=_p(dd.seg_start), uniq=_p(dd.uniq),
                                perm=_p(dd.perm), grad_in=_p(grad_in), g_stride=grad_in.stride(0), Kp=Kp,
                                v=_p(table.v), v_stride=v_stride, w=_p(table.w), w_stride=table.w.stride(0),
                                s0v=_p(table.s0v), s1v=_p(table.s1v), s_stride=s_stride, s0w=_p(table.s0w),
                                s1w=_p(table.s1w), opt_type=opt.code, lr=float(opt.lr), l1=float(opt.l1),
                                l2=float(opt.l2), beta=float(opt.beta), dtype=dt, max_unique=max(dd.n, 1),
                                stream=_stream(grad_in), sr_counter=_p(sr_counter))
    else:
        native.cpu().apply_rows(U=dd.sync(), seg_start=_p(dd.seg_start), uniq=_p(dd.uniq), perm=_p(dd.perm),
                                grad_in=_p(grad_in), g_stride=grad_in.stride(0), Kp=Kp, v=_p(table.v),
                                v_stride=v_stride, w=_p(table.w), w_stride=table.w.stride(0), s0v=_p(table.s0v),
                                s1v=_p(table.s1v), s_stride=s_stride, s0w=_p(table.s0w), s1w=_p(table.s1w),
                                opt_type=opt.code, lr=float(opt.lr), l1=float(opt.l1), l2=float(opt.l2),
                                beta=float(opt.beta), dtype=dt, threads=threads)


def dense_apply(grad: torch.Tensor, table: TableState, opt: OptConfig, Kp: int, row0: int = 0,
                rows: int | None = None, zero: bool = True, sr_counter: torch.Tensor | None = None) -> None:
    """Replicated-table update from a dense gradient buffer ``grad`` [n, Kp+4] (rows
    [g_v | g_w | touch | pad], e.g. all-reduced over the data-parallel ranks): every row whose
    touch word is non-zero gets one optimizer step on table row ``row0 + i`` and (``zero``) is
    cleared for the next step; untouched rows cost one word read.  GPU only; no host sync."""
    _check(_is_gpu(grad), "dense_apply is a GPU path")
    n = grad.shape[0] if rows is None else int(rows)
    v_stride = _chk_rows(table.v, Kp, "v")
    _check(grad.dtype == torch.float32 and grad.is_contiguous() and grad.shape[1] >= Kp + 2
           and grad.shape[1] % 4 == 0, "grad: contiguous fp32 [n, Kp+4]")
    _check(row0 >= 0 and row0 + n <= table.v.shape[0], "dense_apply rows outside the table")
    s_stride = table.s0v.stride(0) if table.s0v is not None else 0
    native.hip().dense_apply(R=n, row0=row0, grad=_p(grad), g_stride=grad.stride(0), touch_col=Kp + 1,
                             zero=int(zero), Kp=Kp, v=_p(table.v), v_stride=v_stride, w=_p(table.w),
                             w_stride=table.w.stride(0), s0v=_p(table.s0v), s1v=_p(table.s1v), s_stride=s_stride,
                             s0w=_p(table.s0w), s1w=_p(table.s1w), opt_type=opt.code, lr=float(opt.lr),
                             l1=float(opt.l1), l2=float(opt.l2), beta=float(opt.beta),
                             dtype=dtype_code(table.v.dtype), stream=_stream(grad), sr_counter=_p(sr_counter))


def zero_listed_rows(buf: torch.Tensor, rows: torch.Tensor, count: torch.Tensor, max_n: int) -> None:
    """buf[rows[i]] = 0 for i < count (device int32 scalar, capped at ``max_n``); GPU, no host sync."""
    _check(_is_gpu(buf) and buf.dtype == torch.float32 and buf.is_contiguous() and buf.shape[1] % 4 == 0,
           "buf: contiguous fp32 rows, width a multiple of 4")
    _chk_vec(rows, torch.int32, None, "rows", buf.device)
    _chk_vec(count, torch.int32, 1, "count", buf.device)
    native.hip().zero_listed_rows(buf=_p(buf), row_words=buf.stride(0), list=_p(rows), count=_p(count),
                                  max_n=int(min(max_n, rows.numel())), stream=_stream(buf))


def apply_runs(req: torch.Tensor, run_off: torch.Tensor, splits: list[int], grad_in: torch.Tensor,
               table: TableState, opt: OptConfig, Kp: int, match: torch.Tensor | None = None,
               threads: int = 0, ws: DedupWorkspace | None = None, grad_bf16: bool = False,
               sr_counter: torch.Tensor | None = None, self_run: int = -1,
               self_excl: torch.Tensor | None = None) -> None:
    """Owner side of a sharded update over the received requests as W ascending runs.

    ``req`` [R] holds the local rows requested by each source rank, rank-major
    (``splits[q]`` rows from rank q, ascending and distinct within a run);
    ``grad_in`` [R, >= Kp+1] the matching gradient rows.  Every distinct row gets
    the sum of its gradient rows in source-rank order and one optimizer step.
    On the GPU the grouping is a cross-run binary-search match (``run_off`` =
    device int32 [W+1] prefix of ``splits``, ``match`` int32 scratch of R*W when
    W > 1) instead of a sort; on the CPU a stable sort of ``req`` (``ws``).
    ``self_run`` >= 0 (GPU): the rows of that run flagged in ``self_excl`` (None: all of them)
    were updated in place by the backward (``SelfRows``) and are skipped.
    """
    R, W = int(sum(splits)), len(splits)
    _chk_vec(req, torch.int32, R, "req", req.device)
    _check(grad_in.dtype == torch.float32 and grad_in.stride(1) == 1 and grad_in.shape[0] >= R, "grad_in: fp32 rows")
    if R == 0:
        return
    if not _is_gpu(grad_in):
        _check(not grad_bf16 and self_run < 0, "bf16 gradient rows and self runs are a GPU path")
        dd = dedup(req[:R], ws=ws, key_bits=32, want_perm=True)
        apply_rows(dd, grad_in, table, opt, Kp, threads=threads)  # (CPU tables: fp32 / bf16, nearest)
        return
    v_stride = _chk_rows(table.v, Kp, "v")
    _range_check(req[:R], table.v.shape[0], "req")
    _chk_vec(run_off, torch.int32, W + 1, "run_off", req.device)
    if W > 1:
        _chk_vec(match, torch.int32, R * W, "match", req.device)
    dt = dtype_code(table.v.dtype)
    s_stride = table.s0v.stride(0) if table.s0v is not None else 0
    native.hip().apply_runs(R=R, W=W, run_off=_p(run_off), req=_p(req), match=_p(match) if W > 1 else 0,
                            grad_in=_p(grad_in), g_stride=grad_in.stride(0), Kp=Kp, v=_p(table.v), v_stride=v_stride,
                            w=_p(table.w), w_stride=table.w.stride(0), s0v=_p(table.s0v), s1v=_p(table.s1v),
                            s_stride=s_stride, s0w=_p(table.s0w), s1w=_p(table.s1w), opt_type=opt.code,
                            lr=float(opt.lr), l1=float(opt.l1), l2=float(opt.l2), beta=float(opt.beta), dtype=dt,
                            stream=_stream(grad_in), g_wcol=(Kp * 2 + 15) // 16 * 4 if grad_bf16 else Kp,
                            g_bf16=int(bool(grad_bf16)), sr_counter=_p(sr_counter), self_run=int(self_run),
                            self_excl=_p(self_excl))


def self_excl(req: torch.Tensor, W: int, run_off: torch.Tensor, me: int, n: int, out: torch.Tensor) -> torch.Tensor:
    """GPU: out[i] = 1 when request ``run_off[me] + i`` (this rank's own run) is in no other run."""
    _chk_vec(out, torch.int32, None, "excl", req.device)
    _check(out.numel() >= n, "excl too short")
    native.hip().self_excl(req=_p(req), W=int(W), run_off=_p(run_off), me=int(me), n=int(n), excl=_p(out),
                           stream=_stream(req))
    return out


@dataclass
class WireFormat:
    """Row layout of the row-sharded exchange (owner gather -> all-to-all -> fwd/bwd).

    A wire row is ``rb`` bytes: the Kp factor values in ``dtype`` (padded to
    ``vb`` bytes), then ``[w, scale, |v|^2, tag]`` fp32 (scale and the stored row norm for fp8 only;
    tag: patch gathers).  bf16 /
    fp8 tables travel at their storage size (the stored bits); an fp32 table
    travels as fp32 (``[v | w | pad]``, the same bytes as a [Kp+4] fp32 row) or,
    with ``comm_dtype = bf16``, as bf16 (rounded to nearest even).
    """

    dtype: torch.dtype
    Kp: int
    vb: int
    rb: int
    table_dtype: torch.dtype
    grad_bf16: bool = False   # gradient rows: [Kp bf16 | pad to gvb][gw fp32, 0, 0, 0] instead of [Kp fp32 | gw | pad]
    g_words: int = 0          # 4-byte words per gradient row
    g_wcol: int = 0           # word index of the w-gradient

    @staticmethod
    def make(table_dtype: torch.dtype, Kp: int, comm_dtype: str = "auto") -> "WireFormat":
        if comm_dtype not in ("auto", "bf16", "fp32", "storage"):
            raise ValueError(f"comm_dtype must be auto|storage|fp32|bf16, got {comm_dtype}")
        dt = table_dtype
        if comm_dtype == "bf16" and table_dtype == torch.float32 and Kp % 8 == 0:
            dt = torch.bfloat16
        if comm_dtype == "fp32":
            dt = torch.float32
        esz = torch.tensor([], dtype=dt).element_size()
        vb = (Kp * esz + 15) // 16 * 16
        gbf = comm_dtype == "bf16"
        gvb = (Kp * 2 + 15) // 16 * 16
        g_words, g_wcol = ((gvb + 16) // 4, gvb // 4) if gbf else (Kp + 4, Kp)
        return WireFormat(dt, Kp, vb, vb + 16, table_dtype, gbf, g_words, g_wcol)

    def empty_grads(self, n: int, device) -> torch.Tensor:
        """Gradient rows in the wire's gradient layout (fp32 words; bf16 pairs packed when ``grad_bf16``)."""
        return torch.empty((n, self.g_words), dtype=torch.float32, device=device)

    @property
    def fp32(self) -> bool:
        return self.dtype == torch.float32

    def empty(self, n: int, device) -> torch.Tensor:
        if self.fp32:
            return torch.empty((n, self.rb // 4), dtype=torch.float32, device=device)
        return torch.empty((n, self.rb), dtype=torch.uint8, device=device)

    def views(self, buf: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """(v [n, Kp] in the wire dtype, w [n] fp32 strided view; fp8 scale at w + 1) of a wire buffer."""
        if self.fp32:
            return buf[:, : self.Kp], buf[:, self.Kp]
        return buf.view(self.dtype)[:, : self.Kp], buf.view(torch.float32)[:, self.vb // 4]


def gather_wire(req: torch.Tensor, table: TableState, fmt: WireFormat, out: torch.Tensor,
                threads: int = 0, idx: torch.Tensor | None = None, run_off: torch.Tensor | None = None,
                W: int = 1, skip: tuple[int, int] | None = None) -> torch.Tensor:
    """Owner side of a sharded lookup: wire rows of table rows ``req`` into ``out`` (``fmt.empty``).

    With ``idx`` (GPU; patch gathers of the early row exchange) row p is ``req[idx[p]]``
    and its last tail word gets the tag ``idx[p] - run_off[run]`` (W ascending runs).
    ``skip`` (GPU, without ``idx``): requests [s0, s1) are left out (self rows)."""
    if fmt.fp32 and table.v.dtype == torch.float32 and idx is None:
        return gather_rows(req, table, fmt.Kp, out, threads=threads, skip=skip)
    _check(skip is None or idx is None, "skip ranges are for plain gathers")
    _check(_is_gpu(req), "non-fp32 wire formats and tagged gathers are a GPU path")
    R = req.numel() if idx is None else idx.numel()
    _chk_vec(req, torch.int32, None, "req", req.device)
    if idx is not None:
        _chk_vec(idx, torch.int32, R, "idx", req.device)
        _chk_vec(run_off, torch.int32, W + 1, "run_off", req.device)
    ok = out.is_contiguous() and out.shape[0] >= R and out.shape[1] * out.element_size() == fmt.rb
    _check(ok and out.dtype in (torch.uint8, torch.float32), "out: [R, rb bytes] wire buffer")
    v = table.v
    _chk_rows(v, fmt.Kp, "v")
    _range_check(req, v.shape[0], "req")
    to_bf16 = v.dtype == torch.float32 and fmt.dtype == torch.bfloat16
    _check(to_bf16 or v.dtype == fmt.dtype, f"wire dtype {fmt.dtype} cannot carry a {v.dtype} table")
    native.hip().gather_wire(R=R, req=_p(req), v=_p(v), v_bytes_stride=v.stride(0) * v.element_size(),
                             w=_p(table.w), w_stride=table.w.stride(0), vbytes=fmt.Kp * v.element_size(),
                             scaled=int(v.dtype == FP8), to_bf16=int(to_bf16), out=_p(out), rb=fmt.rb, vb=fmt.vb,
                             stream=_stream(req), idx=_p(idx), run_off=_p(run_off), W=int(W),
                             skip0=(skip or (0, 0))[0], skip1=(skip or (0, 0))[1])
    return out


def dirty_scan(req: torch.Tensor, run_off: torch.Tensor, W: int, prev: torch.Tensor, prev_off: torch.Tensor,
               Wp: int, flag: torch.Tensor, dcount: torch.Tensor, skip: tuple[int, int] | None = None) -> None:
    """GPU: flag[i] = req[i] in any of the Wp runs of ``prev``; dcount[q] = flagged per run q of ``req``.
    Requests in ``skip`` = [s0, s1) (self rows, read from the table) are never flagged."""
    R = req.numel()
    s0, s1 = skip or (0, 0)
    native.hip().dirty_scan(R=R, req=_p(req), W=int(W), run_off=_p(run_off), Wp=int(Wp), prev_off=_p(prev_off),
                            prev=_p(prev), flag=_p(flag), dcount=_p(dcount), stream=_stream(req), skip0=s0,
                            skip1=s1)


def select_flagged(flag: torch.Tensor, out: torch.Tensor, count: torch.Tensor, ws: torch.Tensor) -> None:
    """GPU stream compaction: out[0..count) = ascending i with flag[i] != 0 (no host sync)."""
    n = flag.numel()
    native.hip().select_flagged(n=n, flag=_p(flag), out=_p(out), count=_p(count), ws=_p(ws), ws_bytes=ws.numel(),
                                stream=_stream(flag))


def select_workspace(n: int, device) -> torch.Tensor:
    return torch.empty(max(native.hip().select_workspace_bytes(max(n, 1)), 1), dtype=torch.uint8, device=device)


def patch_scatter(recv: torch.Tensor, n: int, W: int, recv_off: torch.Tensor, sc_start: torch.Tensor,
                  gathered: torch.Tensor) -> None:
    """GPU: wire row p of ``recv`` (rank-major by owner, ``recv_off``) -> ``gathered[sc_start[owner] + tag]``."""
    rb = recv.shape[1] * recv.element_size()
    native.hip().patch_scatter(D=int(n), recv=_p(recv), rb=rb, W=int(W), recv_off=_p(recv_off),
                               sc_start=_p(sc_start), gathered=_p(gathered), stream=_stream(recv))


# ---------------------------------------------------------------------------
# GPU libsvm tokenizer (hip/parse.hip)
# ---------------------------------------------------------------------------
@dataclass
class ParsedGpu:
    labels: torch.Tensor     # [n] f32
    offsets: torch.Tensor    # [n+1] i32
    ids: torch.Tensor        # [nnz] i32
    vals: torch.Tensor | None  # [nnz] f32, None when every value is 1
    nnz: int
    max_feats: int
    fallback: bool           # syntax outside the GPU subset (or an error): re-parse on the CPU


class ParsePending:
    """A launched GPU tokenizer pass whose (fallback, max_feats, non-unit, nnz) summary is on its
    way to pinned host memory; ``finish()`` waits for it (an event, not a stream sync), so the
    caller can stage and launch the next batch in between."""

    def __init__(self, labels, offsets, ids, vals, info_h, ev):
        self.labels, self.offsets, self.ids, self.vals = labels, offsets, ids, vals
        self.info_h, self.ev = info_h, ev

    def finish(self) -> ParsedGpu:
        self.ev.synchronize()
        info = self.info_h
        fb, mf, nonunit, nnz = int(info[0]), int(info[1]), int(info[2]), int(info[4])
        return ParsedGpu(self.labels, self.offsets, self.ids[:nnz], self.vals[:nnz] if nonunit else None, nnz, mf,
                         bool(fb))


def parse_gpu_start(buf: torch.Tensor, line_start: torch.Tensor, vocab_size: int, hash_feature_id: bool = False,
                    stream: torch.cuda.Stream | None = None, require_vals: bool = False) -> ParsePending:
    """Launch the tokenizer of n '\n'-terminated libsvm lines (``buf`` uint8 on the GPU, line ``i``
    = ``buf[line_start[i]:line_start[i+1]]``) into CSR on the device, asynchronously on
    ``stream``; see ``parse_gpu``."""
    _check(_is_gpu(buf) and buf.dtype == torch.uint8 and buf.is_contiguous(), "buf: uint8 GPU bytes")
    _check(line_start.dtype == torch.int64 and line_start.device == buf.device, "line_start: int64 on buf's device")
    n = line_start.numel() - 1
    dev = buf.device
    st = stream or torch.cuda.current_stream(dev)
    h = native.hip()
    cap = buf.numel() // 2 + n + 1          # a token takes >= 2 bytes (separator + 1 char)
    i32 = dict(dtype=torch.int32, device=dev)
    with torch.cuda.stream(st):
        offsets = torch.empty(n + 1, **i32)
        counts = torch.empty(n + 1, **i32)
        labels = torch.empty(n, dtype=torch.float32, device=dev)
        ids = torch.empty(cap, **i32)
        vals = torch.empty(cap, dtype=torch.float32, device=dev)
        status = torch.empty(5, **i32)
        wsb = h.parse_workspace_bytes(max(n, 1))
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        h.parse(buf=_p(buf), line_start=_p(line_start), n=n, vocab=int(vocab_size), hash=int(bool(hash_feature_id)),
                counts=_p(counts), offsets=_p(offsets), labels=_p(labels), ids=_p(ids), vals=_p(vals),
                status=_p(status), ws=_p(ws), ws_bytes=wsb, stream=st.cuda_stream,
                require_vals=int(bool(require_vals)))
        status[4:5].copy_(offsets[n:])   # (fallback, max_feats, non-unit, -, nnz)
        info_h = torch.empty(5, dtype=torch.int32, pin_memory=True)
        info_h.copy_(status, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
    return ParsePending(labels, offsets, ids, vals, info_h, ev)


def parse_gpu(buf: torch.Tensor, line_start: torch.Tensor, vocab_size: int, hash_feature_id: bool = False,
              stream: torch.cuda.Stream | None = None, require_vals: bool = False) -> ParsedGpu:
    """Tokenize n '\n'-terminated libsvm lines on the GPU (launch + wait, see
    ``parse_gpu_start``).  When ``fallback`` is set the outputs are incomplete and the caller
    must parse the lines with the CPU parser (exact reference semantics and error messages)."""
    return parse_gpu_start(buf, line_start, vocab_size, hash_feature_id, stream, require_vals).finish()


def run_member(req: torch.Tensor, prev: torch.Tensor, prev_run_off: torch.Tensor | None,
               prev_splits: list[int]) -> torch.Tensor:
    """int32 flag per element of ``req``: 1 when the row is in ``prev`` (W ascending runs of
    ``prev_splits`` rows, device offsets ``prev_run_off`` on the GPU), else 0."""
    R = req.numel()
    flag = torch.empty(R, dtype=torch.int32, device=req.device)
    if R == 0:
        return flag
    P = int(sum(prev_splits))
    if not _is_gpu(req):
        return torch.isin(req, prev[:P]).to(torch.int32)
    _chk_vec(req, torch.int32, R, "req", req.device)
    _chk_vec(prev, torch.int32, P, "prev", req.device)
    _chk_vec(prev_run_off, torch.int32, len(prev_splits) + 1, "prev_run_off", req.device)
    native.hip().run_member(R=R, req=_p(req), W=len(prev_splits), run_off=_p(prev_run_off), prev=_p(prev),
                            flag=_p(flag), stream=_stream(req))
    return flag
