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
import weakref

import torch

from ..data.batch import Batch
from ..ops import kernels as K
from ..utils.trace import roctx_range

from .table import FMTable, bits_for, rows_per_shard


def side_stream_priority() -> int:
    """HIP priority of the lookahead / plan streams (FM_SIDE_PRIORITY: 0 = normal, -1 = high).

    The next batch's dedup (+ the sharded plan's owner counts) runs beside this
    step's forward/backward; a high-priority queue lets its small, dependent
    kernels through instead of queueing behind the compute stream's workgroups."""
    return int(os.environ.get("FM_SIDE_PRIORITY", "0"))


def side_stream(device):
    """Stream of the lookahead / plan work (normal queue; FM_SIDE_PRIORITY for its priority).

    Measured alternatives (profiles/README.md): a high-priority queue (no gain) and a
    CU-masked queue restricted to 32-128 CUs (hipExtStreamCreateWithCUMask: 0.67 -> 1.01
    ms/step, the masked queue does not overlap with the compute stream's work)."""
    return torch.cuda.Stream(device, priority=side_stream_priority())


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
    comm_dtype: str = "auto"          # row-sharded wire rows: auto (= storage dtype) | fp32 | bf16
    microbatches: int = 0             # row-sharded step: parts per batch overlapping the exchange (0/1 = one)
    prefetch_rows: str = "auto"       # row-sharded step: early row exchange + patch (auto = on when world > 1)
    overlap_grads: str = "auto"       # row-sharded step: split backward, first half's grads sent early (auto: on)
    staleness: int = 0                # row-sharded step: 0 = synchronous, 1 = bounded staleness (ShardExchange)
    dedup_chunk: int = 32             # CH of the segmented backward
    threads: int = 0                  # CPU kernels (0 = OpenMP default)
    global_bias: bool = False         # learned global bias b0 (extension; the reference has none)
    stochastic_rounding: bool = True  # bf16 / fp8 tables (GPU): stochastically rounded row stores


@dataclass
class StepOut:
    loss_sum: torch.Tensor            # 0-d, summed weighted loss of this rank's batch
    n: int                            # examples in this rank's batch

    def mean_loss(self) -> float:
        return float(self.loss_sum) / max(self.n, 1)


class _Workspace:
    """Per-step buffers, grown on demand and then reused (no per-step allocation)."""

    def __init__(self, device: torch.device, Kp: int, CH: int, r1_dtype: torch.dtype = torch.float32):
        self.device, self.Kp, self.CH, self.r1_dtype = device, Kp, CH, r1_dtype
        self.cap_b = self.cap_n = 0

    def ensure(self, B: int, nnz: int) -> None:
        dev, Kp = self.device, self.Kp
        if B > self.cap_b:
            cap = max(B, int(self.cap_b * 1.25))
            self.pred = torch.empty(cap, dtype=torch.float32, device=dev)
            self.dpred = torch.empty(cap, dtype=torch.float32, device=dev)
            self.r1 = torch.empty((cap, Kp), dtype=self.r1_dtype, device=dev)
            self.cap_b = cap
        if nnz > self.cap_n:
            cap = max(nnz, int(self.cap_n * 1.25), 1)
            self.dd = K.DedupWorkspace(cap, dev, self.CH)
            self.rows32 = torch.empty(cap, dtype=torch.int32, device=dev)
            self.bwd_partial = (torch.empty((K.partial_rows(cap, self.CH), Kp + 4), dtype=torch.float32, device=dev)
                                if dev.type == "cuda" else None)
            self.cap_n = cap
        if not hasattr(self, "fwd_partial"):
            self.fwd_partial = torch.zeros(3 * 4096, dtype=torch.float32, device=dev)

class _LocalSlot:
    """Double-buffered dedup workspace of the local lookahead pipeline."""

    def __init__(self):
        self.dd: K.DedupWorkspace | None = None
        self.rows32: torch.Tensor | None = None
        self.done = None

    def ensure(self, nnz: int, dev, CH: int) -> None:
        if self.dd is None or self.dd.cap < nnz:
            cap = max(nnz, 1, int(1.25 * (self.dd.cap if self.dd else 0)))
            self.dd = K.DedupWorkspace(cap, dev, CH)
            self.rows32 = torch.empty(cap, dtype=torch.int32, device=dev)


@dataclass
class _LocalPlan:
    b: Batch
    slot: int
    rows: torch.Tensor
    dd: object
    ready: object


class _LookaheadGraphRing:
    """hipGraphs of the lookahead local step over a ring of n (even) static input buffers.

    Graph k replays [side stream: csr_rows + dedup of buffer k+1 into slot (k+1)%2]
    concurrently with [main: forward + loss + backward/update of buffer k reading
    slot k%2], i.e. the eager lookahead step with one launch.  The plan of buffer 0
    is built eagerly once; a launch of graph k completes before graph k+1 starts, so
    slot k%2 is never written while it is read.
    """

    def __init__(self, model: "FactorizationMachine", example: Batch, n: int):
        if n < 2 or n % 2:
            raise ValueError("the lookahead ring needs an even number (>= 2) of buffers")
        self.m = weakref.proxy(model)  # no cycle: a dropped model is closed by refcount at once
        dev = model.device

        def static(t):
            return None if t is None else torch.empty_like(t, device=dev)

        ids = example.ids if example.ids.dtype == torch.int32 else example.ids.to(torch.int32)
        self.bufs = [Batch(static(example.labels), static(example.offsets), static(ids), static(example.vals),
                           static(example.weights), example.nnz, max_feats=example.max_feats) for _ in range(n)]
        self.graphs: list = [None] * n
        self.outs: list = [None] * n
        self.dds: list = [None, None]    # DedupOut views of slot 0 / 1 (fixed addresses)
        self.rows: list = [None, None]
        self.primed = False

    def index(self, b: Batch, nb: Batch | None) -> int:
        n = len(self.bufs)
        for k, buf in enumerate(self.bufs):
            if buf.ids.data_ptr() == b.ids.data_ptr():
                return k if nb is not None and self.bufs[(k + 1) % n].ids.data_ptr() == nb.ids.data_ptr() else -1
        return -1

    def _body(self, k: int) -> StepOut:
        m, n = self.m, len(self.bufs)
        main = torch.cuda.current_stream(m.device)
        side = m._side_stream()
        side.wait_stream(main)
        nxt = (k + 1) % n
        with torch.cuda.stream(side):
            self.rows[nxt % 2], self.dds[nxt % 2] = m._plan_into(m._lslots[nxt % 2], self.bufs[nxt])
        out = m._fwd_bwd_local(self.bufs[k], self.rows[k % 2], self.dds[k % 2])
        main.wait_stream(side)
        return out

    def replay(self, k: int) -> StepOut:
        m = self.m
        m.ws.ensure(self.bufs[k].B, self.bufs[k].nnz)
        if not self.primed:  # plan of buffer 0, eagerly
            self.rows[0], self.dds[0] = m._plan_into(m._lslots[0], self.bufs[0])
            self.primed = True
        if self.graphs[k] is None:
            torch.cuda.synchronize(m.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.outs[k] = self._body(k)  # capture executes nothing; the replay below runs the step
            self.graphs[k] = g
        self.graphs[k].replay()
        return StepOut(self.outs[k].loss_sum.clone(), self.bufs[k].B)


class _GraphedStep:
    """A hipGraph of the local training step over static input buffers."""

    def __init__(self, model: "FactorizationMachine", ex: Batch, warmup: int = 1):
        self.m = weakref.proxy(model)
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
        # (dp_dense: the replica is cut into P blocks of W equal row ranges, one per rank)
        rows_multiple = 1
        if mode == "dp_dense":
            from ..parallel.exchange import dp_dense_blocks

            rows_multiple = self.world * dp_dense_blocks(self.world)
        self.table = FMTable(cfg.vocabulary_size, cfg.factor_num, world=self.world if sharded else 1,
                             rank=self.rank if sharded else 0, dtype=cfg.dtype, opt=cfg.opt,
                             init_range=cfg.init_value_range, seed=cfg.seed, device=self.device,
                             rows_multiple=rows_multiple)
        self.K, self.Kp = self.table.K, self.table.Kp
        self.rps = rows_per_shard(cfg.vocabulary_size, self.world) if sharded else cfg.vocabulary_size
        self.ws = _Workspace(self.device, self.Kp, cfg.dedup_chunk, K.r1_dtype(cfg.dtype))
        self.global_step = 0
        self._side = None
        # lookahead dedup plans (eager local path): the current step's plan and up to two pending
        # ones (next batch, and the one after with the depth-2 lookahead) each own a slot
        self._lslots = [_LocalSlot(), _LocalSlot(), _LocalSlot()]
        self._lpending = None
        self._lpending2 = None
        self._llast = 2
        self._ring = None
        self._graph = None
        self._graph_pool: list[_GraphedStep] = []
        self._exchange = None
        # stochastic rounding of low-precision row stores: a device step counter ticked inside
        # every (captured) step, so graph replays draw fresh random bits
        self.sr_base = (cfg.seed * 7919) & 0x3FFFFFFF
        self.sr_state = (torch.full((1,), self.sr_base, dtype=torch.int32, device=self.device)
                         if cfg.stochastic_rounding and cfg.dtype != torch.float32 and self.device.type == "cuda"
                         else None)
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
        self.closed = False
        if self._exchange is not None:  # holds communicators: closed by dist.shutdown() first
            from ..parallel.dist import register_closeable

            register_closeable(self)

    # ------------------------------------------------------------------
    def close(self) -> None:
        """Release the step executor's device resources in a safe order: wait for the
        device, drop captured hipGraphs (their kernel nodes reference workspace and stream
        state), close the exchange (pending RCCL works, its plan communicator), then the
        side / dense streams.  Idempotent; the table stays readable (checkpointing after
        close works), further ``train_step`` calls raise.  ``Trainer`` and
        ``parallel.dist.shutdown()`` call it, so no teardown is left to the garbage
        collector (a communicator finalised by it after the process group was destroyed
        aborted the process: round-1 GPU suite, commit 62c2bac)."""
        if getattr(self, "closed", True):
            return
        self.closed = True
        if self.device.type == "cuda" and torch.cuda.is_initialized():
            torch.cuda.synchronize(self.device)
        for g in ([self._graph] if self._graph is not None else []) + list(self._graph_pool):
            if g.graph is not None:
                g.graph.reset()
            g.graph = None
        if self._ring is not None:
            for g in self._ring.graphs:
                if g is not None:
                    g.reset()
            self._ring.graphs = [None] * len(self._ring.graphs)
        self._graph, self._graph_pool, self._ring = None, [], None
        if self._exchange is not None:
            self._exchange.close()
            self._exchange = None
        self._lpending = self._lpending2 = None
        self._lslots = [_LocalSlot(), _LocalSlot(), _LocalSlot()]
        self._side = None
        if self.device.type == "cuda" and torch.cuda.is_initialized():
            torch.cuda.synchronize(self.device)

    def __del__(self):
        # refcount drop (helpers and exchanges hold the model through weak proxies, so there
        # is no cycle): the teardown runs right where the last reference goes, in program order
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown: HIP / dist may be gone already
            pass

    def __enter__(self) -> "FactorizationMachine":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def sr_tick(self) -> torch.Tensor | None:
        """Advance the stochastic-rounding step counter (on the current stream); its tensor or None."""
        if self.sr_state is None:
            return None
        self.sr_state.add_(1)
        return self.sr_state

    def sr_reset(self) -> None:
        """Re-derive the stochastic-rounding counter from global_step (after a restore)."""
        if self.sr_state is not None:
            self.sr_state.fill_((self.sr_base + self.global_step) & 0x3FFFFFFF)

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
    def train_step(self, b: Batch, next_batch: Batch | None = None, next2: Batch | None = None) -> StepOut:
        """One synchronous training step on ``b``.

        ``next_batch`` / ``next2`` (optional lookahead): the batches of the following
        calls; the executors prepare their table-independent work (dedup, id exchange,
        early row exchange) concurrently with this step."""
        if self.closed:
            raise RuntimeError("train_step on a closed FactorizationMachine")
        if self._ring is not None and (k := self._ring.index(b, next_batch)) >= 0:
            out = self._ring.replay(k)
        elif self._graph is not None and self._graph.matches(b):
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
                out = self._exchange.train_step(b, next_batch, next2)
            elif self._exchange is not None:
                out = self._exchange.train_step(b)
            elif self.device.type == "cuda" and (next_batch is not None or self._lpending is not None):
                out = self._local_lookahead_step(b, next_batch, next2)
            else:
                out = self._local_train_step(b)
        self.global_step += 1
        return out

    def flush(self) -> None:
        """Make every training update visible in the table (bounded-staleness sharded steps apply each
        gradient one step late: the pending one is applied now); no-op otherwise."""
        fl = getattr(self._exchange, "flush", None)
        if fl is not None:
            fl()

    def _side_stream(self):
        if self._side is None:
            self._side = side_stream(self.device)
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
            side = self._side_stream()
            side.wait_stream(main)  # inputs ready; previous step's readers of ws.dd are enqueued before
            with torch.cuda.stream(side), roctx_range("dedup"):
                sb = self._slot_bits(b)
                dd = K.dedup(rows, ws=ws.dd, key_bits=bits_for(self.table.rows), gen_codes=True, vals=b.vals,
                             num_examples=b.B, Kp=self.Kp, ex_shift=sb, offsets=b.offsets)
        else:
            ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz)
        with roctx_range("fwd"):
            fo = K.fm_forward(b.offsets, rows, b.vals, self.table.v, self.table.w, self.Kp, labels=b.labels,
                              weights=b.weights, loss=cfg.loss_type, grad_scale=self.grad_scale(b.B), want_r1=True,
                              pred=ws.pred[: b.B], r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial,
                              threads=cfg.threads, bias=self.gbias, defer_loss=gpu, max_feats=b.max_feats)
            self.bias_step(fo.dpred)
        if gpu:
            main.wait_stream(side)
        else:
            dd = K.dedup(rows, ws=ws.dd, key_bits=bits_for(self.table.rows), ex_of_occ=ex, vals=b.vals)
        rv, rw = self.reg_coeffs
        with roctx_range("bwd+update"):
            K.fm_backward(dd, fo.dpred, fo.r1, self.Kp, mode=K.BWD_LOCAL, table=self.table.state, opt=cfg.opt,
                          reg_v=rv, reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads, sr_counter=self.sr_tick())
        return StepOut(fo.finish_loss(), b.B)

    # ------------------------------------------------------------------
    def _local_plan(self, b: Batch, inputs_ready=None, avoid: int | None = None) -> "_LocalPlan":
        """dedup (+ csr_rows) of ``b`` on the side stream into the next of the plan slots.

        Slots are taken round robin, so the live plans -- the current step's and at most two
        pending ones, the last three created -- never share one; ``slot.done`` orders the reuse
        after the step that last read it.  ``avoid``: the slot of a plan whose step has not
        recorded its ``done`` yet (dp_dense plans ahead before the current step's collectives)."""
        idx = (self._llast + 1) % len(self._lslots)
        if idx == avoid:
            idx = (idx + 1) % len(self._lslots)
        self._llast = idx
        slot = self._lslots[idx]
        cfg = self.cfg
        st = self._side_stream()
        if slot.done is not None:
            st.wait_event(slot.done)       # the step that last read this slot has finished
        ready = getattr(b, "ready", None) or inputs_ready
        if ready is not None:
            st.wait_event(ready)
        else:
            st.wait_stream(torch.cuda.current_stream(self.device))
        for t in (b.labels, b.offsets, b.ids, b.vals, b.weights):
            if t is not None:
                t.record_stream(st)
        with torch.cuda.stream(st), roctx_range("dedup_next"):
            rows, dd = self._plan_into(slot, b)
            ev = torch.cuda.Event()
            ev.record(st)
        return _LocalPlan(b, idx, rows, dd, ev)

    def _plan_into(self, slot: "_LocalSlot", b: Batch):
        """dedup of ``b`` (occurrence codes generated inside its sort) into ``slot`` on the current stream;
        returns (rows, DedupOut)."""
        cfg = self.cfg
        slot.ensure(b.nnz, self.device, cfg.dedup_chunk)
        rows = b.ids if b.ids.dtype == torch.int32 else slot.rows32[: b.nnz].copy_(b.ids)
        sb = self._slot_bits(b)
        kb = bits_for(self.table.rows)
        dd = K.dedup(rows, ws=slot.dd, key_bits=kb, gen_codes=True, vals=b.vals,
                     num_examples=b.B, Kp=self.Kp, ex_shift=sb, offsets=b.offsets)
        return rows, dd

    def _fwd_bwd_local(self, b: Batch, rows: torch.Tensor, dd) -> StepOut:
        """Forward + loss + backward/update of ``b`` on the current stream (dedup ``dd`` ready)."""
        ws, cfg = self.ws, self.cfg
        rv, rw = self.reg_coeffs
        with roctx_range("fwd"):
            fo = K.fm_forward(b.offsets, rows, b.vals, self.table.v, self.table.w, self.Kp, labels=b.labels,
                              weights=b.weights, loss=cfg.loss_type, grad_scale=self.grad_scale(b.B), want_r1=True,
                              pred=ws.pred[: b.B], r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial,
                              threads=cfg.threads, bias=self.gbias, defer_loss=True, max_feats=b.max_feats)
            self.bias_step(fo.dpred)
        with roctx_range("bwd+update"):
            K.fm_backward(dd, fo.dpred, fo.r1, self.Kp, mode=K.BWD_LOCAL, table=self.table.state, opt=cfg.opt,
                          reg_v=rv, reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads,
                          sr_counter=self.sr_tick())
        return StepOut(fo.finish_loss(), b.B)

    def _local_lookahead_step(self, b: Batch, next_batch: Batch | None, next2: Batch | None = None) -> StepOut:
        """Eager local step with lookahead: the dedup of ``next_batch`` runs on the side stream
        concurrently with this step's forward + backward (the dedup of ``b`` was done the same
        way during the previous step), taking the sort off the critical path.  With ``next2``
        (depth-2 lookahead, FM_LOCAL_DEPTH2 != 0) the dedup of the batch after that is started
        too, so a plan has a whole step of slack before its step needs it."""
        ws, cfg = self.ws, self.cfg
        main = torch.cuda.current_stream(self.device)
        nb_ready = None
        if next_batch is not None and getattr(next_batch, "ready", None) is None:
            nb_ready = torch.cuda.Event()   # next_batch's producers: everything enqueued so far
            nb_ready.record(main)
        pl = self._lpending
        if pl is not None and pl.b is b:
            self._lpending, self._lpending2 = self._lpending2, None
        else:
            self._lpending = self._lpending2 = None
            pl = self._local_plan(b)
        main.wait_event(pl.ready)
        out = self._fwd_bwd_local(b, pl.rows, pl.dd)
        done = torch.cuda.Event()
        done.record(main)
        self._lslots[pl.slot].done = done
        if next_batch is not None and (self._lpending is None or self._lpending.b is not next_batch):
            self._lpending = self._local_plan(next_batch, nb_ready)
            self._lpending2 = None
        if (next2 is not None and self._lpending is not None and self._lpending2 is None
                and os.environ.get("FM_LOCAL_DEPTH2", "1") != "0"):
            if getattr(next2, "ready", None) is None and nb_ready is None:
                nb_ready = torch.cuda.Event()
                nb_ready.record(main)
            self._lpending2 = self._local_plan(next2, nb_ready)
        return out

    def lookahead_graph_buffers(self, example: Batch, n: int = 4) -> list[Batch]:
        """Static input buffers of a lookahead hipGraph ring (local GPU step).

        Calling ``train_step(bufs[k], bufs[(k + 1) % n])`` replays graph k: this
        step's forward/backward and, concurrently, the dedup of the next buffer (the
        producer writes batch k+1 into bufs[k+1] before that call)."""
        if self.device.type != "cuda" or self._exchange is not None:
            raise RuntimeError("graph capture is available for the local GPU step")
        self._ring = _LookaheadGraphRing(self, example, n)
        return self._ring.bufs

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
        if self.closed and self.mode != "local":
            raise RuntimeError("forward on a closed multi-rank FactorizationMachine")
        if self._exchange is not None:
            return self._exchange.forward(b, loss=loss, want_reg=want_reg)
        rows = b.ids.to(torch.int32)
        return K.fm_forward(b.offsets, rows, b.vals, self.table.v, self.table.w, self.Kp, labels=b.labels,
                            weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False, want_reg=want_reg,
                            threads=self.cfg.threads, bias=self.gbias, max_feats=b.max_feats)

    def predict(self, b: Batch) -> torch.Tensor:
        """Raw scores (logits for logistic loss), like the reference's pred_ops (run_tffm.py:10-17)."""
        return self.forward(b).pred

    def eval_loss(self, b: Batch) -> float:
        """Weighted mean loss of the configured type (reference valid_op, fm_model.py:317-333)."""
        fo = self.forward(b, loss=self.cfg.loss_type)
        return float(fo.loss_sum) / max(b.B, 1)
