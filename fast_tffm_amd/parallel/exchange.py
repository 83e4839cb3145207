"""Multi-rank step executors (RCCL over xGMI on GPU, gloo on CPU).

Reference communication (all implicit TF gRPC Send/Recv to parameter servers,
SURVEY.md §2.3): C3 = embedding_lookup gather of the batch's unique ids from
the PS-resident ``vocab_block_p`` (partition_strategy "mod",
tffm/fm_model.py:291), C4 = IndexedSlices gradient push + SparseApplyAdagrad on
the PS (fm_model.py:341-348), applied asynchronously per worker.

Replacements here, one process per GPU:

``ShardExchange`` (row-sharded table, the north-star layout): ids are owned
by ``g % world``.  Each rank dedups its batch, sends the unique ids to their
owners with one ``all_to_all_single``, owners gather the rows from HBM and send
them back (second a2a), the fused forward/backward runs on the gathered rows
and emits one gradient row per unique id, a third a2a returns the gradient
rows, and every owner sums the rows it received for the same id (in source-rank
order: deterministic) and applies the optimizer once.  On a fully connected
8-GPU xGMI mesh an all-to-all drives all 7 links of every GPU at once, which is
why lookups/grads use a2a rather than ring collectives.

``DPExchange`` (replicated table, sparse): every rank computes gradient rows for
its unique ids; ids and rows are all-gathered and every rank applies the same
merged update (identical tables by construction, no parameter broadcast).

``DPDenseExchange`` (replicated table, dense): gradient rows are scattered into
a dense ``[vocab, Kp+4]`` buffer that is all-reduced (ring/tree over xGMI);
meant for small vocabularies (BASELINE config 3).
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from ..data.batch import Batch
from ..ops import kernels as K
from ..models.table import bits_for


def make_exchange(model):
    if model.mode == "shard":
        return ShardExchange(model)
    if model.mode == "dp":
        return DPExchange(model)
    if model.mode == "dp_dense":
        return DPDenseExchange(model)
    raise ValueError(model.mode)


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: list[int], in_splits: list[int], group) -> None:
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


class _Base:
    def __init__(self, model):
        self.m = model
        self.ctx = model.dist
        self.group = self.ctx.group
        self.W = model.world
        self.Kp = model.Kp
        self.gs = model.Kp + 4          # exchange row: [v(Kp) | w | pad 3]
        self.dev = model.device
        self.dd2ws: K.DedupWorkspace | None = None

    def _dd2(self, n: int) -> K.DedupWorkspace:
        if self.dd2ws is None or self.dd2ws.cap < n:
            self.dd2ws = K.DedupWorkspace(max(n, 1, int(1.25 * (self.dd2ws.cap if self.dd2ws else 0))), self.dev)
        return self.dd2ws


class ShardExchange(_Base):
    def __init__(self, model):
        super().__init__(model)
        self.Rps = model.rps
        self.key_bits = bits_for(self.W * self.Rps)

    def _keys(self, b: Batch) -> torch.Tensor:
        return K.shard_keys(b.ids, self.W, self.Rps, self.m.ws.rows32)

    def _lookup(self, b: Batch, ex: torch.Tensor | None, sb: int = 0):
        """dedup + a2a(ids) + owner gather + a2a(rows). Returns (dd, gathered, splits, req_recv).

        ``sb`` > 0: ``ex`` holds packed occurrence codes (csr_rows slot_bits)."""
        ws = self.m.ws
        keys = self._keys(b)
        dd = K.dedup(keys, ws=ws.dd, key_bits=self.key_bits, ex_of_occ=ex, vals=b.vals if ex is not None else None,
                     want_inv=True, num_examples=b.B, Kp=self.m.Kp, ex_shift=sb,
                     offsets=b.offsets if sb else None)
        # per-owner counts on the device, one count all-to-all, ONE host sync for both split lists
        counts = torch.empty(2 * self.W, dtype=torch.int64, device=self.dev)
        counts[: self.W] = K.owner_counts(dd, self.Rps, self.W)
        dist.all_to_all_single(counts[self.W:], counts[: self.W], group=self.group)
        both = counts.tolist()
        sc, rc = both[: self.W], both[self.W:]
        U = int(sum(sc))
        dd.U_host = U
        R = int(sum(rc))
        uniq = dd.uniq[:U]
        req_send = torch.remainder(uniq, self.Rps)  # keys are owner * Rps + local row
        req_recv = torch.empty(R, dtype=torch.int32, device=self.dev)
        _a2a(req_recv, req_send, rc, sc, self.group)
        rows_send = torch.empty((R, self.gs), dtype=torch.float32, device=self.dev)
        K.gather_rows(req_recv, self.m.table.state, self.Kp, rows_send, threads=self.m.cfg.threads)
        gathered = torch.empty((U, self.gs), dtype=torch.float32, device=self.dev)
        _a2a(gathered, rows_send, sc, rc, self.group)
        return dd, gathered, (sc, rc), req_recv

    def train_step(self, b: Batch):
        from ..models.fm import StepOut

        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        sb = m._slot_bits(b, always=True)
        ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz, slot_bits=sb)
        dd, gathered, (sc, rc), req_recv = self._lookup(b, ex, sb)
        U = dd.U_host
        R = req_recv.numel()
        # owner side: group the received requests by table row now, on a side stream,
        # concurrently with this rank's forward/backward (it only needs req_recv)
        gpu = self.dev.type == "cuda"
        if gpu:
            main = torch.cuda.current_stream(self.dev)
            side = m._side_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dd2 = K.dedup(req_recv, ws=self._dd2(R), key_bits=bits_for(self.Rps), want_perm=True)
        else:
            dd2 = K.dedup(req_recv, ws=self._dd2(R), key_bits=bits_for(self.Rps), want_perm=True)
        src_v, src_w = gathered[:, :Kp], gathered[:, Kp]
        fo = K.fm_forward(b.offsets, dd.inv[: b.nnz], b.vals, src_v, src_w, Kp, labels=b.labels,
                          weights=b.weights, loss=cfg.loss_type, grad_scale=m.grad_scale(b.B), want_r1=True,
                          pred=ws.pred[: b.B], r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial,
                          threads=cfg.threads)
        grad = torch.empty((U, self.gs), dtype=torch.float32, device=self.dev)
        rv, rw = m.reg_coeffs
        K.fm_backward(dd, fo.dpred, fo.r1, Kp, mode=K.BWD_EMIT, src_v=src_v, src_w=src_w, grad_out=grad, reg_v=rv,
                      reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads)
        grad_recv = torch.empty((R, self.gs), dtype=torch.float32, device=self.dev)
        _a2a(grad_recv, grad, rc, sc, self.group)
        if gpu:
            main.wait_stream(side)
        K.apply_rows(dd2, grad_recv, m.table.state, cfg.opt, Kp, threads=cfg.threads)
        return StepOut(fo.loss_sum, b.B)

    @torch.no_grad()
    def forward(self, b: Batch, *, loss: str = "none", want_reg: bool = False) -> K.FwdOut:
        self.m.ws.ensure(b.B, b.nnz)
        dd, gathered, _, _ = self._lookup(b, None)
        return K.fm_forward(b.offsets, dd.inv[: b.nnz], b.vals, gathered[:, : self.Kp], gathered[:, self.Kp],
                            self.Kp, labels=b.labels, weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False,
                            want_reg=want_reg, threads=self.m.cfg.threads)


class DPExchange(_Base):
    """Replicated table; sparse all-gather of (ids, gradient rows)."""

    def _local_grads(self, b: Batch):
        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        rows = m._rows32(b)
        ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz)
        fo = K.fm_forward(b.offsets, rows, b.vals, m.table.v, m.table.w, Kp, labels=b.labels, weights=b.weights,
                          loss=cfg.loss_type, grad_scale=m.grad_scale(b.B), want_r1=True, pred=ws.pred[: b.B],
                          r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial, threads=cfg.threads)
        dd = K.dedup(rows, ws=ws.dd, key_bits=bits_for(m.table.rows), ex_of_occ=ex, vals=b.vals,
                     num_examples=b.B, Kp=Kp)
        U = dd.sync()
        uniq = dd.uniq[:U]
        src = torch.empty((U, self.gs), dtype=torch.float32, device=self.dev)
        K.gather_rows(uniq, m.table.state, Kp, src, threads=cfg.threads)
        grad = torch.empty((U, self.gs), dtype=torch.float32, device=self.dev)
        rv, rw = m.reg_coeffs
        K.fm_backward(dd, fo.dpred, fo.r1, Kp, mode=K.BWD_EMIT, src_v=src[:, :Kp], src_w=src[:, Kp],
                      grad_out=grad, reg_v=rv, reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads)
        return fo, uniq, grad

    def train_step(self, b: Batch):
        from ..models.fm import StepOut

        fo, uniq, grad = self._local_grads(b)
        U = uniq.numel()
        sizes_t = torch.tensor([U], dtype=torch.int64, device=self.dev)
        sizes = [torch.empty_like(sizes_t) for _ in range(self.W)]
        dist.all_gather(sizes, sizes_t, group=self.group)
        sizes = [int(s.item()) for s in sizes]
        umax = max(max(sizes), 1)
        ids_pad = torch.zeros(umax, dtype=torch.int32, device=self.dev)
        ids_pad[:U] = uniq
        g_pad = torch.zeros((umax, self.gs), dtype=torch.float32, device=self.dev)
        g_pad[:U] = grad
        ids_all = [torch.empty_like(ids_pad) for _ in range(self.W)]
        g_all = [torch.empty_like(g_pad) for _ in range(self.W)]
        dist.all_gather(ids_all, ids_pad, group=self.group)
        dist.all_gather(g_all, g_pad, group=self.group)
        ids_cat = torch.cat([ids_all[r][: sizes[r]] for r in range(self.W)])
        g_cat = torch.cat([g_all[r][: sizes[r]] for r in range(self.W)])
        n = ids_cat.numel()
        dd2 = K.dedup(ids_cat, ws=self._dd2(n), key_bits=bits_for(self.m.table.rows), want_perm=True)
        K.apply_rows(dd2, g_cat, self.m.table.state, self.m.cfg.opt, self.Kp, threads=self.m.cfg.threads)
        return StepOut(fo.loss_sum, b.B)

    @torch.no_grad()
    def forward(self, b: Batch, *, loss: str = "none", want_reg: bool = False) -> K.FwdOut:
        t = self.m.table
        return K.fm_forward(b.offsets, b.ids.to(torch.int32), b.vals, t.v, t.w, self.Kp, labels=b.labels,
                            weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False, want_reg=want_reg,
                            threads=self.m.cfg.threads)


class DPDenseExchange(DPExchange):
    """Replicated table; dense all-reduce of a [vocab, Kp+4] gradient buffer (small vocabularies)."""

    def __init__(self, model):
        super().__init__(model)
        V = model.table.rows
        self.dense = torch.zeros((V, self.gs), dtype=torch.float32, device=self.dev)
        self.arange = torch.arange(V + 1, dtype=torch.int32, device=self.dev)

    def train_step(self, b: Batch):
        from ..models.fm import StepOut

        fo, uniq, grad = self._local_grads(b)
        dense = self.dense
        dense.zero_()
        idx = uniq.to(torch.int64)
        dense.index_copy_(0, idx, grad)
        dense[idx, self.Kp + 1] = 1.0  # touch counter travels in a pad column
        dist.all_reduce(dense, group=self.group)
        touched = torch.nonzero(dense[:, self.Kp + 1] > 0).flatten().to(torch.int32)
        T = touched.numel()
        dd = K.DedupOut(n=T, uniq=touched, perm=touched, seg_start=self.arange[: T + 1],
                        num_unique=torch.tensor([T], dtype=torch.int32, device=self.dev), U_host=T)
        K.apply_rows(dd, dense, self.m.table.state, self.m.cfg.opt, self.Kp, threads=self.m.cfg.threads)
        return StepOut(fo.loss_sum, b.B)
