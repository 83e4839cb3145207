"""The factorization machine and its fused training step.

Reference behaviour (tffm/fm_model.py:267-365): embedding_lookup of the unique
ids -> FmScorer -> loss (mean of weighted logistic/MSE) -> Adagrad.minimize of
``loss + reg_score / batch_size`` (``batch_size`` = the configured one).

Here the step is an explicit pipeline of native kernels, no autograd graph:

  local (world == 1):   fwd+loss (direct table gather) | dedup -> bwd+optimizer
  shard (row-sharded):  dedup -> a2a(ids) -> owner gather -> a2a(rows) -> fwd
                        -> bwd(emit grads) -> a2a(grads) -> owner sum+optimizer
  dp    (replicated):   local fwd/bwd(emit) -> all_gather(ids, grads) -> every
                        rank applies the identical merged update
  dp_dense:             dense all_reduce of a [vocab, Kp+4] gradient buffer

The reference trains asynchronously (between-graph replication, no
SyncReplicasOptimizer: run_tffm.py:204-211); these modes are synchronous SPMD.
``grad_reduce = sum`` (default) adds every rank's mean-loss gradient, which is
what W asynchronous workers apply per W steps; ``mean`` divides by W.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import os

import torch

from ..data.batch import Batch
from ..ops import kernels as K
from ..utils.trace import roctx_range

# dedup on a side stream concurrently with the forward (1) or before it on the same stream (0)
_SIDE_STREAM = os.environ.get("FM_SIDE_STREAM", "1") == "1"
from .table import FMTable, bits_for, rows_per_shard


@dataclass
class FMConfig:
    vocabulary_size: int
    factor_num: int
    loss_type: str = "mse"            # "mse" | "logistic"
    factor_lambda: float = 0.0
    bias_lambda: float = 0.0
    batch_size: int = 50000           # configured batch size: reg_score / batch_size (fm_model.py:345-347)
    init_value_range: float = 0.01
    seed: int = 0
    dtype: torch.dtype = torch.float32
    opt: K.OptConfig = field(default_factory=K.OptConfig)
    mode: str = "auto"                # auto | local | shard | dp | dp_dense
    grad_reduce: str = "sum"          # sum | mean (multi-rank)
    dedup_chunk: int = 32             # CH of the segmented backward
    threads: int = 0                  # CPU kernels (0 = OpenMP default)
    global_bias: bool = False         # learned global bias b0 (extension; the reference has none)


@dataclass
class StepOut:
    loss_sum: torch.Tensor            # 0-d, summed weighted loss of this rank's batch
    n: int                            # examples in this rank's batch

    def mean_loss(self) -> float:
        return float(self.loss_sum) / max(self.n, 1)


class _Workspace:
    """Per-step buffers, grown on demand and then reused (no per-step allocation)."""

    def __init__(self, device: torch.device, Kp: int, CH: int):
        self.device, self.Kp, self.CH = device, Kp, CH
        self.cap_b = self.cap_n = 0

    def ensure(self, B: int, nnz: int) -> None:
        dev, Kp = self.device, self.Kp
        if B > self.cap_b:
            cap = max(B, int(self.cap_b * 1.25))
            self.pred = torch.empty(cap, dtype=torch.float32, device=dev)
            self.dpred = torch.empty(cap, dtype=torch.float32, device=dev)
            self.r1 = torch.empty((cap, Kp), dtype=torch.float32, device=dev)
            self.cap_b = cap
        if nnz > self.cap_n:
            cap = max(nnz, int(self.cap_n * 1.25), 1)
            self.dd = K.DedupWorkspace(cap, dev, self.CH)
            self.rows32 = torch.empty(cap, dtype=torch.int32, device=dev)
            self.bwd_partial = (torch.empty((K.partial_rows(cap, self.CH), Kp + 4), dtype=torch.float32, device=dev)
                                if dev.type == "cuda" else None)
            self.cap_n = cap
        if not hasattr(self, "dense_part"):
            self.dense_part = (torch.empty((K.DENSE_WG * K.MAX_DENSE, Kp + 4), dtype=torch.float32, device=dev)
                               if dev.type == "cuda" and Kp <= 128 else None)
        if not hasattr(self, "fwd_partial"):
            self.fwd_partial = torch.zeros(3 * 4096, dtype=torch.float32, device=dev)


class _GraphedStep:
    """A hipGraph of the local training step over static input buffers."""

    def __init__(self, model: "FactorizationMachine", ex: Batch, warmup: int = 1):
        self.m = model
        dev = model.device
        self.sig = self._sig(ex)

        def static(t):
            return None if t is None else torch.empty_like(t, device=dev)

        ids = ex.ids if ex.ids.dtype == torch.int32 else ex.ids.to(torch.int32)
        self.inp = Batch(static(ex.labels), static(ex.offsets), static(ids), static(ex.vals), static(ex.weights),
                         ex.nnz, max_feats=ex.max_feats)
        self.eager_left = max(1, warmup)  # real (eager) steps before capture: lazy loads, workspace sizing
        self.graph = None
        self.out = None

    def _capture(self) -> None:
        dev = self.m.device
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self.m._local_train_step(self.inp)

    @staticmethod
    def _sig(b: Batch):
        return (b.B, b.nnz, b.vals is not None, b.weights is not None, FactorizationMachine._slot_bits(b))

    def matches(self, b: Batch) -> bool:
        return self._sig(b) == self.sig

    def owns(self, b: Batch) -> bool:
        return b.ids.data_ptr() == self.inp.ids.data_ptr() and b.offsets.data_ptr() == self.inp.offsets.data_ptr()

    def _load(self, b: Batch) -> None:
        for dst, src in ((self.inp.labels, b.labels), (self.inp.offsets, b.offsets), (self.inp.ids, b.ids),
                         (self.inp.vals, b.vals), (self.inp.weights, b.weights)):
            if dst is not None and src is not None and dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)

    def replay(self, b: Batch) -> StepOut:
        if self.eager_left > 0:
            self.eager_left -= 1
            self.m.ws.ensure(b.B, b.nnz)
            return self.m._local_train_step(b)
        self._load(b)
        if self.graph is None:
            self._capture()  # capture does not execute: the replay below runs this step
        self.graph.replay()
        return StepOut(self.out.loss_sum.clone(), b.B)


class FactorizationMachine:
    """FM model + step executor for one rank."""

    def __init__(self, cfg: FMConfig, device: torch.device | str = "cpu", dist=None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dist = dist
        self.world = dist.world if dist is not None else 1
        self.rank = dist.rank if dist is not None else 0
        mode = cfg.mode
        if mode == "auto":
            mode = "local" if self.world == 1 else "shard"
        if mode == "local" and self.world > 1:
            raise ValueError("mode=local needs world_size == 1")
        self.mode = mode
        sharded = mode == "shard"
        self.table = FMTable(cfg.vocabulary_size, cfg.factor_num, world=self.world if sharded else 1,
                             rank=self.rank if sharded else 0, dtype=cfg.dtype, opt=cfg.opt,
                             init_range=cfg.init_value_range, seed=cfg.seed, device=self.device)
        self.K, self.Kp = self.table.K, self.table.Kp
        self.rps = rows_per_shard(cfg.vocabulary_size, self.world) if sharded else cfg.vocabulary_size
        self.ws = _Workspace(self.device, self.Kp, cfg.dedup_chunk)
        self.global_step = 0
        self._side = None
        self._graph = None
        self._graph_pool: list[_GraphedStep] = []
        self._exchange = None
        # optional global bias b0 (+ optimizer state), replicated on every rank; its gradient
        # sum(dpred) is all-reduced over the ranks each step (the model's one dense parameter)
        if cfg.global_bias:
            acc0 = float(cfg.opt.initial_accumulator) if cfg.opt.name in ("adagrad", "ftrl") else 0.0
            self.gbias = torch.zeros(1, dtype=torch.float32, device=self.device)
            self.gbias_s0 = torch.full((1,), acc0, dtype=torch.float32, device=self.device)
            self.gbias_s1 = torch.zeros(1, dtype=torch.float32, device=self.device)
        else:
            self.gbias = self.gbias_s0 = self.gbias_s1 = None
        if mode in ("shard", "dp", "dp_dense") and self.world >= 1 and dist is not None:
            from ..parallel.exchange import make_exchange

            self._exchange = make_exchange(self)
        elif mode != "local":
            raise ValueError(f"mode={mode} needs a distributed context")

    # ------------------------------------------------------------------
    @property
    def reg_coeffs(self) -> tuple[float, float]:
        """(lambda_f, lambda_b) / configured batch size: d(reg_score / batch_size)/d(params) scale."""
        s = 1.0 / float(self.cfg.batch_size)
        if self.world > 1 and self.cfg.grad_reduce == "mean":
            s /= self.world
        return self.cfg.factor_lambda * s, self.cfg.bias_lambda * s

    def grad_scale(self, B: int) -> float:
        s = 1.0 / max(B, 1)
        if self.world > 1 and self.cfg.grad_reduce == "mean":
            s /= self.world
        return s

    def bias_step(self, dpred: torch.Tensor) -> None:
        """Update the global bias from this rank's dpred (dL/dpred, already scaled): the
        gradient sum(dpred) is summed over ranks (all-reduce), then the optimizer step
        (same rule as the table's) runs identically on every rank.  Graph-capturable."""
        if self.gbias is None:
            return
        g = dpred.sum().reshape(1)
        if self.dist is not None and self.world > 1:
            import torch.distributed as tdist

            tdist.all_reduce(g, group=self.dist.group)
        o = self.cfg.opt
        if o.name == "adagrad":
            self.gbias_s0.add_(g * g)
            self.gbias.sub_(o.lr * g * torch.rsqrt(self.gbias_s0))
        elif o.name == "ftrl":
            n_new = self.gbias_s0 + g * g
            self.gbias_s1.add_(g - (n_new.sqrt() - self.gbias_s0.sqrt()) / o.lr * self.gbias)
            self.gbias_s0.copy_(n_new)
            quad = (o.beta + n_new.sqrt()) / o.lr + 2.0 * o.l2
            z = self.gbias_s1
            self.gbias.copy_(torch.where(z.abs() > o.l1, (torch.sign(z) * o.l1 - z) / quad, torch.zeros_like(z)))
        else:
            self.gbias.sub_(o.lr * g)

    @staticmethod
    def _slot_bits(b: Batch, always: bool = False) -> int:
        """Packed occurrence codes (csr_rows slot_bits) for GPU batches whose dedup needs the
        occurrence index (per-occurrence values, or ``always``: the sharded inverse map)."""
        if b.ids.device.type != "cuda" or not (always or b.vals is not None):
            return 0
        return K.slot_bits_for(b.B, b.max_feats)

    def _rows32(self, b: Batch) -> torch.Tensor:
        if b.ids.dtype == torch.int32:
            return b.ids
        out = self.ws.rows32[: b.nnz]
        out.copy_(b.ids)  # int64 -> int32 (ids < vocabulary_size < 2^31)
        return out

    # ------------------------------------------------------------------
    def train_step(self, b: Batch, next_batch: Batch | None = None) -> StepOut:
        """One synchronous training step on ``b``.

        ``next_batch`` (optional lookahead): the batch of the following call;
        multi-rank executors prepare its table-independent work (dedup, id
        exchange) concurrently with this step."""
        if self._graph is not None and self._graph.matches(b):
            g = self._graph
            # a batch that already lives in a captured graph's input buffers replays that graph, no copy
            for other in self._graph_pool:
                if other.owns(b):
                    g = other
                    break
            out = g.replay(b)
        else:
            self.ws.ensure(b.B, b.nnz)
            if getattr(self._exchange, "supports_lookahead", False):
                out = self._exchange.train_step(b, next_batch)
            elif self._exchange is not None:
                out = self._exchange.train_step(b)
            else:
                out = self._local_train_step(b)
        self.global_step += 1
        return out

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def _local_train_step(self, b: Batch) -> StepOut:
        """fwd+loss on the current stream, concurrently with dedup on a side stream, then bwd+update.

        The two branches only share read-only inputs; the join is an event, so
        the step stays asynchronous (and graph-capturable).
        """
        ws, cfg = self.ws, self.cfg
        rows = self._rows32(b)
        gpu = self.device.type == "cuda"
        if gpu:
            main = torch.cuda.current_stream(self.device)
            side = self._side_stream() if _SIDE_STREAM else main
            if side is not main:  # (a stream waiting on itself inside a hipGraph capture faults at replay)
                side.wait_stream(main)  # inputs ready; previous step's readers of ws.dd are enqueued before
            with torch.cuda.stream(side), roctx_range("dedup"):
                sb = self._slot_bits(b)
                ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz, slot_bits=sb)
                dd = K.dedup(rows, ws=ws.dd, key_bits=bits_for(self.table.rows), ex_of_occ=ex, vals=b.vals,
                             num_examples=b.B, Kp=self.Kp, ex_shift=sb, offsets=b.offsets,
                             dense_min=K.dense_min_for(b.B, self.Kp, cfg.dedup_chunk))
        else:
            ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz)
        with roctx_range("fwd"):
            fo = K.fm_forward(b.offsets, rows, b.vals, self.table.v, self.table.w, self.Kp, labels=b.labels,
                              weights=b.weights, loss=cfg.loss_type, grad_scale=self.grad_scale(b.B), want_r1=True,
                              pred=ws.pred[: b.B], r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial,
                              threads=cfg.threads, bias=self.gbias)
            self.bias_step(fo.dpred)
        if gpu:
            if side is not main:
                main.wait_stream(side)
        else:
            dd = K.dedup(rows, ws=ws.dd, key_bits=bits_for(self.table.rows), ex_of_occ=ex, vals=b.vals)
        rv, rw = self.reg_coeffs
        with roctx_range("bwd+update"):
            K.fm_backward(dd, fo.dpred, fo.r1, self.Kp, mode=K.BWD_LOCAL, table=self.table.state, opt=cfg.opt,
                          reg_v=rv, reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads, dense_part=ws.dense_part,
                          dense_stream=self._side_stream() if gpu and _SIDE_STREAM else None)
        return StepOut(fo.loss_sum, b.B)

    # ------------------------------------------------------------------
    def capture_graph(self, example: Batch, warmup: int = 1) -> None:
        """Arm hipGraph execution of the local training step for batches shaped like ``example``.

        The next ``warmup`` matching ``train_step`` calls run eagerly; the one
        after captures the step (capture executes nothing) and every matching
        call from then on copies its batch into the graph's static buffers and
        replays the whole step (~10 kernels + the stream fork/join) with one
        launch.  Results are identical to eager execution.
        """
        if self.device.type != "cuda" or self._exchange is not None:
            raise RuntimeError("graph capture is available for the local GPU step")
        self._graph = _GraphedStep(self, example, warmup)

    def graph_input_buffers(self, n: int = 1) -> list[Batch]:
        """Static input batches of ``n`` captured graphs (after ``capture_graph``).

        A producer that writes batches straight into these buffers (e.g. the H2D
        copy of a staging pipeline) replays the matching graph with no extra
        device copy.  The first buffer set belongs to the main graph.
        """
        if self._graph is None:
            raise RuntimeError("call capture_graph first")
        while len(self._graph_pool) < n - 1:
            g = _GraphedStep(self, self._graph.inp, 0)
            g.eager_left = 0
            self._graph_pool.append(g)
        return [self._graph.inp] + [g.inp for g in self._graph_pool[: n - 1]]

    # ------------------------------------------------------------------
    @torch.no_grad()
    def forward(self, b: Batch, *, loss: str = "none", want_reg: bool = False) -> K.FwdOut:
        """Scores (and optionally the summed loss) without touching parameters."""
        if self._exchange is not None:
            return self._exchange.forward(b, loss=loss, want_reg=want_reg)
        rows = b.ids.to(torch.int32)
        return K.fm_forward(b.offsets, rows, b.vals, self.table.v, self.table.w, self.Kp, labels=b.labels,
                            weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False, want_reg=want_reg,
                            threads=self.cfg.threads, bias=self.gbias)

    def predict(self, b: Batch) -> torch.Tensor:
        """Raw scores (logits for logistic loss), like the reference's pred_ops (run_tffm.py:10-17)."""
        return self.forward(b).pred

    def eval_loss(self, b: Batch) -> float:
        """Weighted mean loss of the configured type (reference valid_op, fm_model.py:317-333)."""
        fo = self.forward(b, loss=self.cfg.loss_type)
        return float(fo.loss_sum) / max(b.B, 1)
