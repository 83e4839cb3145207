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

import os
import weakref

import numpy as np
import torch
import torch.distributed as dist

from ..data.batch import Batch
from ..ops import kernels as K
from ..models.table import bits_for
from ..utils.trace import roctx_range


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
        self.m = weakref.proxy(model)   # the model owns the exchange (no reference cycle)
        self.ctx = model.dist
        self.group = self.ctx.group
        self.W = model.world
        self.Kp = model.Kp
        self.gs = model.Kp + 4          # exchange row: [v(Kp) | w | pad 3]
        self.dev = model.device
        self.dd2ws: K.DedupWorkspace | None = None
        # payload bytes this rank has put on the wire to OTHER ranks (collective inputs, counted
        # on the host from the split sizes it already knows; bench.py reports the per-step mean)
        self.bytes_sent = 0

    def _to_others(self, splits: list[int]) -> int:
        """Items of an all-to-all split list that leave this rank."""
        me = self.ctx.rank
        return int(sum(s for q, s in enumerate(splits) if q != me))

    def close(self) -> None:
        """Release device resources (model.close() calls this after a device sync)."""
        self.dd2ws = None

    def _dd2(self, n: int) -> K.DedupWorkspace:
        if self.dd2ws is None or self.dd2ws.cap < n:
            self.dd2ws = K.DedupWorkspace(max(n, 1, int(1.25 * (self.dd2ws.cap if self.dd2ws else 0))), self.dev)
        return self.dd2ws


class _Part:
    """One micro-batch of a sharded step: its examples, dedup grouping, owner split
    sizes and the rows it requests from every owner."""

    __slots__ = ("b", "e0", "dd", "sc", "rc", "U", "R", "u0", "r0", "req_send", "keys", "seg")


class _ShardPlan:
    """The table-independent half of one batch's sharded step: per micro-batch part
    the dedup, owner counts and id all-to-all, plus the owner-side run offsets
    over all parts' received requests (``req_recv`` holds part 0's runs, then
    part 1's, ...; ``run_off`` the W * parts run boundaries)."""

    __slots__ = ("b", "slot", "parts", "U", "R", "req_recv", "run_off", "splits", "match", "ready", "early",
                 "train", "counts", "counts_ev", "self_u", "self_r", "self_excl", "sb", "pieces")


class _Early:
    """Rows of a plan gathered and exchanged ahead of time (during the previous step),
    plus what must be re-sent once the previous step's update has landed: the requests
    (rows) that the previous step also updated -- "dirty" -- with their index in their
    source's run (the tag), per-source counts both ways, and the requester-side base
    position of every patch row it will receive."""

    # GPU: gathered, didx, sc_start, dsend (pinned [2, W]: sent / received dirty counts), ev, work,
    # rows_send; CPU reference: gathered, dirty_rows, dtags, dsend, dpos
    __slots__ = ("gathered", "dirty_rows", "dtags", "dsend", "dpos", "didx", "sc_start", "ev", "work", "rows_send")


class _PlanSlot:
    """Double-buffered device workspaces of a plan (a plan for batch t+1 is built
    while step t still reads the buffers of plan t)."""

    def __init__(self):
        self.dd: list[K.DedupWorkspace | None] = []
        self.keys: list[torch.Tensor | None] = []
        self.dd2: K.DedupWorkspace | None = None   # CPU owner grouping
        self.done: torch.cuda.Event | None = None  # main-stream event: last step using this slot finished
        self.run_off_h: torch.Tensor | None = None  # pinned receive-run offsets (host staging)
        self.run_off: torch.Tensor | None = None    # device copy
        self.match: torch.Tensor | None = None      # [R, runs] cross-run match scratch (apply_runs)
        self.excl: torch.Tensor | None = None       # [own requests] exclusive flags (self rows)
        self.segidx: list[torch.Tensor | None] = []  # per part: key-bucket index (K.seg_index)

    def segidx_buf(self, k: int) -> torch.Tensor | None:
        """Bucket-index buffer of part k (K.seg_index), sized for the workspace's capacity."""
        d = self.dd[k]
        nb = K.seg_index_bits(d.cap, 31)[1]
        while len(self.segidx) <= k:
            self.segidx.append(None)
        if self.segidx[k] is None or self.segidx[k].numel() < nb + 1:
            self.segidx[k] = torch.empty(nb + 1, dtype=torch.int32, device=d.uniq.device)
        return self.segidx[k]

    def ensure(self, k: int, nnz: int, dev, CH: int) -> K.DedupWorkspace:
        while len(self.dd) <= k:
            self.dd.append(None)
            self.keys.append(None)
        d = self.dd[k]
        if d is None or d.cap < nnz:
            cap = max(nnz, 1, int(1.25 * (d.cap if d else 0)))
            self.dd[k] = K.DedupWorkspace(cap, dev, CH)
            self.keys[k] = torch.empty(cap, dtype=torch.int32, device=dev)
        return self.dd[k]

    def runs(self, splits: list[int], dev) -> torch.Tensor:
        """Device int32 prefix offsets of the receive runs, staged through pinned memory.

        Called after this stream's host sync on the owner counts, so the previous
        copy out of the pinned buffer (same stream, earlier) has completed."""
        n = len(splits)
        if self.run_off is None or self.run_off.numel() < n + 1:
            self.run_off_h = torch.empty(n + 1, dtype=torch.int32, pin_memory=True)
            self.run_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
        h = self.run_off_h.numpy()
        h[0] = 0
        np.cumsum(splits, out=h[1: n + 1])
        self.run_off[: n + 1].copy_(self.run_off_h[: n + 1], non_blocking=True)
        return self.run_off

    def excl_buf(self, n: int, dev) -> torch.Tensor:
        if self.excl is None or self.excl.numel() < n:
            self.excl = torch.empty(max(n, 1, int(1.25 * (self.excl.numel() if self.excl is not None else 0))),
                                    dtype=torch.int32, device=dev)
        return self.excl

    def match_buf(self, n: int, dev) -> torch.Tensor:
        if self.match is None or self.match.numel() < n:
            self.match = torch.empty(max(n, 1, int(1.25 * (self.match.numel() if self.match is not None else 0))),
                                     dtype=torch.int32, device=dev)
        return self.match

    def early_ws(self, R: int, W: int, dev) -> dict:
        """Buffers of the early row exchange (device scratch, pinned staging), grown on demand."""
        ew = getattr(self, "_early", None)
        if ew is None or ew["R"] < R or ew["W"] != W:
            cap = max(R, 1, int(1.25 * (ew["R"] if ew else 0)))
            i32 = dict(dtype=torch.int32, device=dev)
            ew = dict(R=cap, W=W, flag=torch.empty(cap, **i32), didx=torch.empty(cap, **i32),
                      dcount=torch.empty(W + 1, **i32), sel=K.select_workspace(cap, dev),
                      drecv=torch.empty(W, **i32),
                      dsend_h=torch.empty((2, W), dtype=torch.int32, pin_memory=True),
                      sc_h=torch.empty(W, dtype=torch.int32, pin_memory=True), sc=torch.empty(W, **i32))
            self._early = ew
        return ew

    def ensure2(self, n: int, dev) -> K.DedupWorkspace:
        if self.dd2 is None or self.dd2.cap < n:
            self.dd2 = K.DedupWorkspace(max(n, 1, int(1.25 * (self.dd2.cap if self.dd2 else 0))), dev)
        return self.dd2


def _sub_batch(b: Batch, e0: int, e1: int, n0: int, n1: int, offsets: torch.Tensor) -> Batch:
    """Examples [e0, e1) of ``b`` (occurrences [n0, n1)) as views, with rebased ``offsets``."""
    return Batch(b.labels[e0:e1], offsets, b.ids[n0:n1], None if b.vals is None else b.vals[n0:n1],
                 None if b.weights is None else b.weights[e0:e1], n1 - n0, max_feats=b.max_feats)


class ShardExchange(_Base):
    N_TRAIN_SLOTS = 3
    EVAL_SLOT = 3

    """Row-sharded step.

    ``train_step(b, next_batch)`` builds the plan of the next batch (everything that
    does not read the table: dedup, counts + id a2a with its one host sync,
    owner-side run offsets) on a side stream while this step's forward/backward
    run, so only gather -> a2a(rows) -> fwd -> bwd -> a2a(grads) -> apply stay on
    the critical path.  Synchronous semantics are unchanged: the rows of step t+1
    are gathered after step t's update.

    With ``microbatches = P > 1`` the batch is cut into P parts with their own
    dedup: the row all-to-all of part k+1 runs on RCCL's stream while part k
    computes, and part k's gradient all-to-all while part k+1 computes; the owner
    sums all parts' gradient rows (P*W runs, fixed order) and applies the
    optimizer once.  Cost: rows used by several parts cross the wire once per
    part (~+20% rows for P=2 on Criteo-shaped batches), the backward runs on
    smaller groups and the plan chain (P dedups) grows: measured at world 1
    (profiles/shard_mb), P=2 adds ~160 us of compute and ~35% to the plan chain,
    more than it can hide when the exchange is link-bound (every a2a shares one
    RCCL stream), so the default is one part.
    """

    supports_lookahead = True

    def __init__(self, model):
        super().__init__(model)
        self.Rps = model.rps
        self.key_bits = bits_for(self.W * self.Rps)
        # training plans rotate over slots 0..2 (current, next, next-but-one); slot 3 belongs to
        # evaluation / prediction plans (forward()), which never reuse a training slot
        self.slots = [_PlanSlot(), _PlanSlot(), _PlanSlot(), _PlanSlot()]
        # wire format of the gathered rows: storage dtype (exact) or bf16 for fp32 tables on request
        tdt = model.table.v.dtype
        self.wire = K.WireFormat.make(tdt, self.Kp, model.cfg.comm_dtype if self.dev.type == "cuda" else "fp32")
        mb = int(getattr(model.cfg, "microbatches", 0) or 0)
        self.nparts = max(1, mb)
        # early row exchange (exact): rows of step t+1 are gathered and exchanged while step t
        # computes; after step t's update only the rows it touched are re-sent (patch)
        pr = str(getattr(model.cfg, "prefetch_rows", "auto")).lower()
        forced = pr in ("on", "true", "1")
        self.prefetch = self.nparts == 1 and (forced or (pr == "auto" and self.W > 1))
        # with only one batch of lookahead the early exchange sits at the end of the plan chain
        # (which can then become the critical path): "auto" uses it with two batches of lookahead
        self.prefetch_depth1 = self.prefetch and forced
        # split backward: the gradient rows of every owner's first half travel (P2P on RCCL)
        # while the second half is reduced, hiding half of the gradient exchange behind compute.
        # "auto" = on with one part at world > 1; off at world 1, where no gradient row leaves the
        # rank and the second pass only costs (k128 fp8 FTRL EMIT 1.121 -> 1.056 ms without it,
        # profiles/README.md round 4; "on" forces it, the tests' way to run the pieces at world 1)
        og = str(getattr(model.cfg, "overlap_grads", "auto")).lower()
        self.overlap_grads = self.nparts == 1 and (og in ("on", "true", "1") or (og == "auto" and self.W > 1))
        # self rows (hip/fm_common.h SelfRows): this rank's own rows are read from the table by the
        # forward / backward -- no owner gather, no row exchange or early copy to patch for them --
        # and the exclusive ones (requested by no other rank this step) are updated in place by
        # the backward instead of the owner's apply.  GPU, wire dtype = table dtype, one part.
        self.self_rows = (self.dev.type == "cuda" and self.wire.dtype == tdt and self.nparts == 1
                          and os.environ.get("FM_SELF_ROWS", "1") != "0")
        # world 1 with self rows: every row is this rank's and exclusive and a key is its table
        # row (owner 0), so a training step IS the local step -- the model's own executor runs it
        # (its dedup lookahead, the fused in-place backward: no plan, gradient rows or apply; the
        # table is the local table) -- as dp_dense does at world 1 (profiles/r4/shard_w1_local.txt);
        # world > 1 keeps EMIT + the exchange
        self.local_w1 = (self.self_rows and self.W == 1
                         and os.environ.get("FM_SHARD_W1_LOCAL", "1") != "0")  # (0: EMIT path, A/B)
        # Bounded staleness (FMConfig.staleness = 1): the reference trains asynchronously -- workers push
        # their sparse gradients to the parameter servers without waiting for each other and read
        # whatever the servers hold (run_tffm.py:204-211, fm_model.py:345-348).  Made deterministic here:
        # step t reads EVERY row (own rows included) as the table is with the gradients of steps <= t-2
        # applied, gathered from the owners and exchanged during step t-1 (no dirty-row patch); step t's
        # gradient all-to-all and the owners' apply run on their own streams beside step t+1's compute
        # (the apply of step t-1 between the gather of step t+1's rows and the apply of step t).  The
        # compute stream never touches the table, so no own-row shortcut (self rows, in-place updates)
        # and no split backward.  Equal to one process applying each step's merged gradient one step late
        # (tests/test_staleness.py).  0 = synchronous (default).
        self.staleness = int(getattr(model.cfg, "staleness", 0) or 0)
        if self.staleness not in (0, 1):
            raise ValueError(f"staleness must be 0 or 1, got {self.staleness}")
        if self.staleness:
            if self.nparts != 1:
                raise ValueError("staleness = 1 runs one part per batch (microbatches <= 1)")
            self.self_rows = self.local_w1 = self.overlap_grads = False
            self.prefetch = True
        self._pend = None             # staleness: (plan, gradient rows, works, sr seed, bwd event) to apply
        self.applied_ev = None        # staleness: the last enqueued apply (apply stream)
        self._gather_ev = None        # staleness: the last gather of a step's rows (the next apply follows it)
        self._apply_st = None
        self._ded = None
        self._main = None             # the compute stream of the current step (starvation check)
        self.host_blocks = self.starved_waits = 0
        self.host_wait_s = 0.0
        self.cur_plan: _ShardPlan | None = None
        self.step_start = None
        self.early_steps = 0          # steps that took the early-exchange + patch path
        # Communicators.  "dual" (default): lookahead plans talk on their own communicator (own
        # RCCL stream), so the id all-to-all of batch t+1 does not queue behind step t's row /
        # grad all-to-alls.  Ordering invariant that keeps this deadlock-free: every rank issues
        # the collectives of EACH communicator in the same host program order (the executor's
        # control flow depends only on values that are identical on all ranks: the lookahead
        # depth and the exchanged count matrices), and the two communicators never wait on each
        # other inside a collective -- a main-communicator collective may depend on a plan
        # collective only through stream events recorded after it on the same rank.  RCCL
        # kernels of the two communicators then make progress independently (each occupies a
        # few CUs).  FM_SINGLE_COMM=1 ("single") routes every collective through the main
        # communicator in program order (no cross-communicator progress assumption; the plan's
        # exchanges then serialise with the step's row / grad all-to-alls).
        single = os.environ.get("FM_SINGLE_COMM", "0") == "1"
        # (FM_COMM_MODE=dual forces the plan communicator at world 1: teardown tests)
        forced = os.environ.get("FM_COMM_MODE", "")
        # dual needs the RCCL streams of both communicators on hardware queues of their own
        # (dist.ensure_hw_queues); with fewer queues (GPU_MAX_HW_QUEUES forced low by the user)
        # every collective goes through the main communicator in program order
        from .dist import MIN_HW_QUEUES, hw_queues

        few_queues = hw_queues() < MIN_HW_QUEUES   # (the count HIP started with, not the env's now)
        self.comm_mode = forced if forced in ("single", "dual") else (
            "single" if (single or self.W == 1 or few_queues) else "dual")
        self.plan_group = (dist.new_group(ranks=list(range(self.W)), backend=dist.get_backend(self.group))
                           if self.comm_mode == "dual" else self.group)
        self.cpu_group = self.ctx.cpu_group or self.group
        self.last_slot = self.N_TRAIN_SLOTS - 1
        self.pending: list[_ShardPlan] = []   # built plans of upcoming batches, in order
        self._prep = None

    def close(self) -> None:
        """Wait for in-flight exchange works, drop every plan (device buffers, pinned
        staging, events) and destroy the plan communicator (dual mode) while the main
        process group is still alive.  With staleness the pending gradient is applied first (the table
        stays complete and readable after close)."""
        if self.staleness and self._pend is not None:
            self.flush()
        for pl in [self.cur_plan] + list(self.pending):
            e = getattr(pl, "early", None) if pl is not None else None
            if e is not None and getattr(e, "work", None) is not None:
                e.work.wait()
                e.work = None
        if self.dev.type == "cuda" and torch.cuda.is_initialized():
            torch.cuda.synchronize(self.dev)
        self.pending, self.cur_plan, self.step_start = [], None, None
        self.slots = [_PlanSlot() for _ in self.slots]
        if self.comm_mode == "dual" and self.plan_group is not None and dist.is_initialized():
            dist.destroy_process_group(self.plan_group)
        self.plan_group = None
        self._prep = self._apply_st = self._ded = self._main = None
        self.applied_ev = self._gather_ev = None
        super().close()

    def _prep_stream(self):
        """Stream of the plan finish (id all-to-all, run offsets, early row exchange)."""
        if self._prep is None:
            from ..models.fm import side_stream

            self._prep = side_stream(self.dev)
        return self._prep

    def _dedup_stream(self):
        """Stream of the plan start (dedup, owner counts, count exchange): its own, so the next plan's
        dedup never queues behind this plan's early row gather, which waits for the previous step's
        update (one stream for both tied the count read of plan t+2 to step t's start)."""
        if self._ded is None:
            from ..models.fm import side_stream

            self._ded = side_stream(self.dev)
        return self._ded

    def _await(self, ev) -> None:
        """Host read of a plan's device-produced counts (pinned copy behind ``ev``).  Normally the event
        finished long ago (no wait).  Otherwise the host blocks -- back-pressure when the host is more
        than a step ahead, counted in ``host_blocks`` -- and, if the compute stream has run dry while the
        host waits, in ``starved_waits`` (a host wait on the critical path)."""
        if ev.query():
            return
        self.host_blocks += 1
        main = self._main
        if main is not None and main.query():
            self.starved_waits += 1
        import time

        t0 = time.perf_counter()
        ev.synchronize()
        self.host_wait_s += time.perf_counter() - t0

    def _split(self, b: Batch, nparts: int) -> list[tuple[int, int, int, int]]:
        """(e0, e1, n0, n1) example / occurrence ranges of the micro-batches of ``b``."""
        if nparts <= 1 or b.B < 2 * nparts:
            return [(0, b.B, 0, b.nnz)]
        cuts = [b.B * i // nparts for i in range(nparts + 1)]
        nz = [0] + [b.host_offset(c) for c in cuts[1:-1]] + [b.nnz]
        return [(cuts[i], cuts[i + 1], nz[i], nz[i + 1]) for i in range(nparts)]

    def _plan(self, b: Batch, train: bool, inputs_ready=None, early: bool = True) -> _ShardPlan:
        """Build the whole plan of ``b`` now (start + finish)."""
        pl = self._plan_start(b, train, inputs_ready)
        self._plan_finish(pl, early)
        return pl

    def _side_ctx(self):
        if self.dev.type == "cuda":
            return torch.cuda.stream(self._prep_stream())
        import contextlib

        return contextlib.nullcontext()

    def _plan_start(self, b: Batch, train: bool, inputs_ready=None) -> _ShardPlan:
        """First half of a plan, host-asynchronous (side stream on the GPU): dedup of every part
        and the per-owner counts, copied to pinned host memory behind an event.  The host does
        not wait for this dedup; ``_plan_finish`` reads the counts one call later.

        ``inputs_ready``: main-stream event after which ``b``'s tensors are valid
        (default: everything enqueued on the current stream so far)."""
        m = self.m
        if train:
            # round robin over the training slots: never the slot of a pending (not yet consumed)
            # plan or of the current step's plan; the last step that used the slot is waited for
            # (done event)
            busy = {p.slot for p in self.pending}
            if self.cur_plan is not None:
                busy.add(self.cur_plan.slot)
            idx = self.last_slot
            for _ in range(self.N_TRAIN_SLOTS):
                idx = (idx + 1) % self.N_TRAIN_SLOTS
                if idx not in busy:
                    break
            else:
                raise RuntimeError("ShardExchange: every training plan slot is in use")
            self.last_slot = idx
        else:
            idx = self.EVAL_SLOT  # (its done event orders it after the previous forward)
        slot = self.slots[idx]
        pl = _ShardPlan()
        pl.b, pl.slot, pl.train = b, idx, train
        pl.early = pl.splits = pl.run_off = pl.match = pl.ready = None
        pl.self_u = pl.self_r = pl.self_excl = pl.sb = pl.pieces = None
        gpu = self.dev.type == "cuda"
        if gpu:
            st = self._dedup_stream()
            if slot.done is not None:
                st.wait_event(slot.done)      # the last step that used these buffers is over
            ready = getattr(b, "ready", None) or inputs_ready
            if ready is not None:
                st.wait_event(ready)           # H2D copy of the batch (Prefetcher) / its producer
            else:
                st.wait_stream(torch.cuda.current_stream(self.dev))
            for t in (b.labels, b.offsets, b.ids, b.vals, b.weights):
                if t is not None:
                    t.record_stream(st)
        ranges = self._split(b, self.nparts if train else 1)
        with (torch.cuda.stream(st) if gpu else self._side_ctx()):
            pl.parts = []
            counts = []
            if gpu:
                # [0] = sent counts, [1] = received counts (world 1: written by owner_counts too), [W, P]
                both = torch.empty((2, self.W, len(ranges)), dtype=torch.int64, device=self.dev)
            for k, (e0, e1, n0, n1) in enumerate(ranges):
                part = _Part()
                offs = b.offsets[e0:e1 + 1] if n0 == 0 else b.offsets[e0:e1 + 1] - n0
                part.b = sb = b if len(ranges) == 1 else _sub_batch(b, e0, e1, n0, n1, offs)
                part.e0 = e0
                dws = slot.ensure(k, sb.nnz, self.dev, m.cfg.dedup_chunk)
                keys, sids = slot.keys[k][: sb.nnz], sb.ids  # sharded keys: written by the dedup's sort
                shift = m._slot_bits(sb, always=True) if train else 0
                # training plans on the GPU find each occurrence's segment through a bucket index
                # (K.seg_index) instead of the inverse map, a 5.1M-occurrence random scatter
                lookup = train and gpu and K.seg_lookup_enabled()
                part.keys = keys
                # (training: occurrence codes generated inside the sort -- csr_rows fused)
                part.dd = K.dedup(keys, ws=dws, key_bits=self.key_bits, gen_codes=train,
                                  vals=sb.vals if train else None, want_inv=not lookup,
                                  num_examples=sb.B, Kp=self.m.Kp, ex_shift=shift,
                                  offsets=sb.offsets if train else None, shard_ids=sids, shard=(self.W, self.Rps))
                part.seg = K.seg_index(part.dd, self.key_bits, slot.segidx_buf(k)) if lookup else None
                if gpu:  # column k of [W, P]: row q = what goes to rank q
                    K.owner_counts(part.dd, self.Rps, self.W, out=both[0, :, k],
                                   out2=both[1, :, k] if self.W == 1 else None)
                else:
                    counts.append(K.owner_counts(part.dd, self.Rps, self.W))
                pl.parts.append(part)
            if gpu:
                # the count exchange runs on the device (RCCL, plan communicator) right behind the
                # dedup, both copied to pinned memory (no stack / copy kernels on the plan's chain)
                if self.W > 1:
                    dist.all_to_all_single(both[1], both[0], group=self.plan_group)
                pl.counts = torch.empty(both.shape, dtype=torch.int64, pin_memory=True)
                pl.counts.copy_(both, non_blocking=True)
                pl.counts_ev = torch.cuda.Event()
                pl.counts_ev.record(st)
            else:
                pl.counts, pl.counts_ev = torch.stack(counts, dim=1), None
        return pl

    def _plan_finish(self, pl: _ShardPlan, early: bool = False) -> None:
        """Second half of a plan: per-owner counts to the host (its dedup finished long ago when
        the plan was started a call earlier), count exchange on the CPU group, id all-to-all,
        owner-side run offsets and -- optionally -- the early row exchange; records ``ready``."""
        if pl.splits is not None:
            return
        gpu = self.dev.type == "cuda"
        slot = self.slots[pl.slot]
        with self._side_ctx():
            if pl.counts_ev is not None:  # GPU: both count matrices exchanged on the device
                self._prep_stream().wait_event(pl.counts_ev)  # (the dedup stream's outputs)
                self._await(pl.counts_ev)
                sc, rc = pl.counts[0].clone(), pl.counts[1].clone()
            else:
                sc = pl.counts.clone()
                if self.W == 1:
                    rc = sc
                else:
                    rc = torch.empty_like(sc)
                    dist.all_to_all_single(rc, sc, group=self.cpu_group)
            sc_l, rc_l = sc.t().tolist(), rc.t().tolist()
            u_off = r_off = 0
            for k, part in enumerate(pl.parts):
                part.sc, part.rc = sc_l[k], rc_l[k]
                part.U, part.R = int(sum(part.sc)), int(sum(part.rc))
                part.u0, part.r0 = u_off, r_off
                u_off += part.U
                r_off += part.R
                part.dd.U_host = part.U
                if K.debug_checks():
                    self._check_splits(part)
            pl.U, pl.R = u_off, r_off
            pl.req_recv = torch.empty(max(pl.R, 1), dtype=torch.int32, device=self.dev)
            for part in pl.parts:
                # keys are owner * Rps + local row: the local rows requested from each owner
                dst = pl.req_recv[part.r0: part.r0 + part.R]
                if self.W == 1:
                    torch.remainder(part.dd.uniq[: part.U], self.Rps, out=dst)  # identity exchange
                else:
                    req_send = torch.remainder(part.dd.uniq[: part.U], self.Rps)
                    _a2a(dst, req_send, part.rc, part.sc, self.plan_group)
                    self.bytes_sent += 4 * self._to_others(part.sc) + 8 * 2 * (self.W - 1) * len(pl.parts)
            # owner-side grouping of the received requests (W * P ascending runs): device
            # run offsets + match scratch for apply_runs; the CPU path sorts inside apply_runs
            pl.splits = [c for part in pl.parts for c in part.rc]
            if pl.train and gpu:
                pl.run_off = slot.runs(pl.splits, self.dev)
                pl.match = slot.match_buf(pl.R * len(pl.splits), self.dev) if len(pl.splits) > 1 else None
                part = pl.parts[0]
                if self.self_rows and len(pl.parts) == 1:
                    me = self.ctx.rank
                    s0, r0 = int(sum(part.sc[:me])), int(sum(part.rc[:me]))
                    pl.self_u, pl.self_r = (s0, s0 + part.sc[me]), (r0, r0 + part.rc[me])
                    if self.W > 1 and part.rc[me]:
                        pl.self_excl = K.self_excl(pl.req_recv, self.W, pl.run_off, me, part.rc[me],
                                                   slot.excl_buf(part.rc[me], self.dev))
            if pl.train and self._split_ok(pl, None):
                self._split_plan(pl)
            if early and pl.train and self._early_ok(pl, self.cur_plan):
                pl.early = self._early(pl, self.cur_plan)
            if gpu:
                pl.ready = torch.cuda.Event()
                pl.ready.record(self._prep_stream())

    def _early_ok(self, pl: _ShardPlan, cur: _ShardPlan | None) -> bool:
        gpu = self.dev.type == "cuda"
        if self.staleness:  # (no dirty scan against the current plan: every row is read stale)
            return pl.train and len(pl.parts) == 1 and pl.splits is not None and (pl.run_off is not None or not gpu)
        if pl.self_r is not None and pl.self_r[1] - pl.self_r[0] == pl.R:
            return False  # every request is this rank's own row (world 1): nothing to exchange early
        return (self.prefetch and len(pl.parts) == 1 and pl.splits is not None and cur is not None
                and cur.splits is not None and (cur.run_off is not None or not gpu) and len(cur.parts) == 1
                and (pl.run_off is not None or not gpu))

    def _early(self, pl: _ShardPlan, cur: _ShardPlan) -> _Early:
        if self.staleness:
            return self._early_stale(pl)
        return self._early_gpu(pl, cur) if self.dev.type == "cuda" else self._early_cpu(pl, cur)

    # ---- bounded staleness -------------------------------------------------------------------
    def _note_gather(self) -> None:
        """Staleness: the gather of a step's rows was enqueued on the current stream; the next apply
        (step t-1's, when these are step t's rows) must follow it."""
        if self.dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self._gather_ev = ev

    def _early_stale(self, pl: _ShardPlan) -> _Early:
        """Staleness: every row ``pl`` requests (own rows included), gathered from the table as it is after
        the apply enqueued last -- step t-1's, when ``pl`` is step t+1's plan -- and before the next one,
        and exchanged now, on the plan stream and communicator; no dirty rows, no patch."""
        dev, W = self.dev, self.W
        gpu = dev.type == "cuda"
        part = pl.parts[0]
        e = _Early()
        e.work = e.rows_send = e.didx = e.sc_start = e.dsend = e.ev = None
        if gpu and self.applied_ev is not None:
            self._prep_stream().wait_event(self.applied_ev)
        rows_send = self.wire.empty(pl.R, dev)
        K.gather_wire(pl.req_recv[: pl.R], self.m.table.state, self.wire, rows_send, threads=self.m.cfg.threads)
        self._note_gather()
        if W == 1:
            e.gathered = rows_send
            return e
        e.gathered = self.wire.empty(pl.U, dev)
        if gpu:
            e.rows_send = rows_send
            e.work = dist.all_to_all_single(e.gathered, rows_send, part.sc, part.rc, group=self.plan_group,
                                            async_op=True)
        else:
            _a2a(e.gathered, rows_send, part.sc, part.rc, self.plan_group)
        self.bytes_sent += self.wire.rb * self._to_others(part.rc)
        return e

    def _apply_stream(self):
        if self._apply_st is None:
            from ..models.fm import side_stream

            self._apply_st = side_stream(self.dev)
        return self._apply_st

    def _apply_pending(self) -> None:
        """Staleness: enqueue the owners' apply of the pending (previous step's) gradient rows on the apply
        stream, behind the last gather of a step's rows (they keep the table as it was before this apply)
        and behind the gradient all-to-all; its event gates the next gather and the plan slot's reuse."""
        p, self._pend = self._pend, None
        if p is None:
            return
        pl, grad_recv, works, sr, bwd_ev = p
        m, cfg = self.m, self.m.cfg
        gpu = self.dev.type == "cuda"
        if gpu:
            st = self._apply_stream()
            cm = torch.cuda.stream(st)
        else:
            import contextlib

            cm = contextlib.nullcontext()
        with cm:
            if gpu:
                st.wait_event(bwd_ev)                # (world 1: no all-to-all orders it after the backward)
                if self._gather_ev is not None:
                    st.wait_event(self._gather_ev)
            for w in works:
                w.wait()                             # GPU: this stream waits for the communicator's
            with roctx_range("apply_stale"):
                K.apply_runs(pl.req_recv, pl.run_off, pl.splits, grad_recv, m.table.state, cfg.opt, self.Kp,
                             match=pl.match, threads=cfg.threads,
                             ws=self.slots[pl.slot].ensure2(pl.R, self.dev) if not gpu else None,
                             grad_bf16=self.wire.grad_bf16, sr_counter=sr, self_run=-1, self_excl=None)
            if gpu:
                for t in (grad_recv, pl.req_recv) + ((sr,) if sr is not None else ()):
                    t.record_stream(st)
                ev = torch.cuda.Event()
                ev.record(st)
                self.applied_ev = ev
                self.slots[pl.slot].done = ev        # (the plan's run offsets / match scratch were read)

    def flush(self) -> None:
        """Staleness: apply the pending gradient now and make the current stream wait for it -- the table
        then holds every step's update (evaluation, checkpoints, teardown).  A step whose rows were not
        gathered yet (no lookahead) then reads them as fresh as a synchronous step would.  No-op when
        synchronous."""
        if not self.staleness:
            return
        self._apply_pending()
        if self.dev.type == "cuda" and self.applied_ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(self.applied_ev)

    def sync_state(self) -> None:
        """Checkpoint hook (utils/checkpoint.py): every update applied."""
        self.flush()

    def _train_step_stale(self, b: Batch, next_batch: Batch | None = None, next2: Batch | None = None):
        """One bounded-staleness step (see __init__).  Host order: take this step's plan (its rows were
        gathered and sent during the previous step, or are gathered now without lookahead), apply the
        previous step's gradient (apply stream), forward + backward on the exchanged rows only, gradient
        all-to-all (pending: applied during the next step), then the next plans and the next step's rows
        (gathered right behind the apply just enqueued)."""
        from ..models.fm import StepOut

        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        gpu = self.dev.type == "cuda"
        wf = self.wire
        build = next2 if next2 is not None else next_batch
        nb_ready = None
        if build is not None and gpu and getattr(build, "ready", None) is None:
            nb_ready = torch.cuda.Event()
            nb_ready.record(self._main)
        with roctx_range("plan"):
            pl = self._take_plan(b, True)
        self.cur_plan = pl
        part = pl.parts[0]
        with roctx_range("rows"):
            if pl.early is not None:
                e = pl.early
                if e.work is not None:
                    e.work.wait()
                    e.work = e.rows_send = None
                buf = e.gathered
                self.early_steps += 1
            else:  # (no lookahead: gathered now, after the last apply and before the pending one)
                if gpu and self.applied_ev is not None:
                    self._main.wait_event(self.applied_ev)
                buf, work = self._gather_part(pl, part, async_op=True)
                self._note_gather()
                if work is not None:
                    work.wait()
        self._apply_pending()  # step t-1's gradient (after the gather of this step's rows)
        src_v, src_w = wf.views(buf)
        grad_send = wf.empty_grads(max(pl.U, 1), self.dev)
        grad_recv = grad_send if self.W == 1 else wf.empty_grads(max(pl.R, 1), self.dev)
        rv, rw = m.reg_coeffs
        sr = m.sr_tick()
        if sr is not None:
            sr = sr.clone()  # (this step's seed, read by its apply during the next step)
        sb, dd = part.b, part.dd
        with roctx_range("fwd"):
            fo = K.fm_forward(sb.offsets, part.keys if part.seg is not None else dd.inv[: sb.nnz], sb.vals, src_v,
                              src_w, Kp, labels=sb.labels, weights=sb.weights, loss=cfg.loss_type,
                              grad_scale=m.grad_scale(b.B), want_r1=True, pred=ws.pred[: sb.B], r1=ws.r1[: sb.B],
                              dpred=ws.dpred[: sb.B], partial=ws.fwd_partial, threads=cfg.threads, bias=m.gbias,
                              seg_lookup=part.seg, defer_loss=True)
        with roctx_range("bwd"):
            K.fm_backward(dd, fo.dpred, fo.r1, Kp, mode=K.BWD_EMIT, src_v=src_v, src_w=src_w,
                          grad_out=grad_send[: max(pl.U, 1)], reg_v=rv, reg_w=rw, partial=ws.bwd_partial,
                          threads=cfg.threads, grad_bf16=wf.grad_bf16)
        m.bias_step(ws.dpred[: b.B])
        loss = fo.finish_loss()
        works, bwd_ev = [], None
        if gpu:
            bwd_ev = torch.cuda.Event()
            bwd_ev.record(self._main)
        if self.W > 1:
            with roctx_range("a2a_grads"):
                works.append(dist.all_to_all_single(grad_recv[: pl.R], grad_send[: pl.U], part.rc, part.sc,
                                                    group=self.group, async_op=True))
                self.bytes_sent += 4 * wf.g_words * self._to_others(part.sc)
        self._pend = (pl, grad_recv, works, sr, bwd_ev)
        # the next plans; the next step's rows are gathered behind the apply enqueued above
        if self.pending and next_batch is not None and self.pending[0].b is next_batch:
            nxt_pl = self.pending[0]
            with roctx_range("plan_finish_next"):
                self._plan_finish(nxt_pl)
            if nxt_pl.early is None and self._early_ok(nxt_pl, pl):
                with roctx_range("early_rows_next"):
                    self._early_ahead(nxt_pl, pl)
        if next2 is not None and not any(p.b is next2 for p in self.pending):
            if next_batch is not None and not any(p.b is next_batch for p in self.pending):
                with roctx_range("plan_next"):
                    self.pending.append(self._plan(next_batch, True, nb_ready, early=True))
            with roctx_range("plan_next2"):
                self.pending.append(self._plan_start(next2, True, nb_ready))
        elif next2 is None and next_batch is not None and not any(p.b is next_batch for p in self.pending):
            with roctx_range("plan_next"):
                self.pending.append(self._plan(next_batch, True, nb_ready, early=True))
        return StepOut(loss, b.B)

    def _early_ahead(self, pl: _ShardPlan, cur: _ShardPlan) -> None:
        """Depth-2 pipeline: at the start of step t, the early row exchange of the (already
        built) plan of step t+1 against step t's plan, on the plan stream; its ready event
        moves past the early work."""
        gpu = self.dev.type == "cuda"
        with self._side_ctx():
            pl.early = self._early(pl, cur)
            if gpu:
                pl.ready = torch.cuda.Event()
                pl.ready.record(self._prep_stream())

    def _patch(self, pl: _ShardPlan) -> tuple[torch.Tensor, torch.Tensor]:
        return self._patch_gpu(pl) if self.dev.type == "cuda" else self._patch_cpu(pl)

    def _early_gpu(self, pl: _ShardPlan, cur: _ShardPlan) -> _Early:
        """GPU version of ``_early_cpu``: one scan kernel (membership + per-source dirty counts),
        a rocPRIM compaction of the dirty positions, an async D2H of the counts, then the early
        gather + row all-to-all -- no host sync and no per-element torch ops."""
        dev, W = self.dev, self.W
        part = pl.parts[0]
        R, U = pl.R, pl.U
        req = pl.req_recv[:R]
        slot = self.slots[pl.slot]
        e = _Early()
        ew = slot.early_ws(R, W, dev)             # this slot's buffers (free again two plans later)
        flag, e.didx, dcount = ew["flag"], ew["didx"], ew["dcount"]  # dcount: [W] per source, [W] total
        K.dirty_scan(req, pl.run_off, W, cur.req_recv, cur.run_off, len(cur.splits), flag, dcount, skip=pl.self_r)
        K.select_flagged(flag[:R], e.didx, dcount[W:], ew["sel"])
        # dirty counts: sent (per source rank) and received (per owner), exchanged on the device
        drecv = ew["drecv"]
        if W == 1:
            drecv.copy_(dcount[:W])
        else:
            dist.all_to_all_single(drecv, dcount[:W], group=self.plan_group)
        e.dsend = ew["dsend_h"]
        e.dsend[0].copy_(dcount[:W], non_blocking=True)
        e.dsend[1].copy_(drecv, non_blocking=True)
        e.ev = torch.cuda.Event()
        e.ev.record(self._prep_stream())
        h = ew["sc_h"].numpy()
        h[0] = 0
        np.cumsum(part.sc[:-1], out=h[1:W])
        e.sc_start = ew["sc"]
        e.sc_start.copy_(ew["sc_h"], non_blocking=True)
        if self.step_start is not None:
            self._prep_stream().wait_event(self.step_start)
        rows_send = self.wire.empty(R, dev)
        K.gather_wire(req, self.m.table.state, self.wire, rows_send, threads=self.m.cfg.threads, skip=pl.self_r)
        e.work = None
        if W == 1:
            e.gathered = rows_send
        else:
            # asynchronous: the plan stream goes on (next dedup) while the rows travel; the
            # compute stream waits for this work before it patches / reads the rows
            e.gathered = self.wire.empty(U, dev)
            e.rows_send = rows_send
            e.work = dist.all_to_all_single(e.gathered, rows_send, part.sc, part.rc, group=self.plan_group,
                                            async_op=True)
            self.bytes_sent += self.wire.rb * self._to_others(part.rc)
        return e

    def _patch_gpu(self, pl: _ShardPlan) -> tuple[torch.Tensor, torch.Tensor]:
        """GPU version of ``_patch_cpu``: one tagged gather of the dirty rows, the patch
        all-to-all, one scatter kernel into the early copies."""
        e, dev, W = pl.early, self.dev, self.W
        self._await(e.ev)  # dirty counts (sent, received) on the host -- long done by now
        ds, dr = e.dsend[0].tolist(), e.dsend[1].tolist()
        D, Dr = int(sum(ds)), int(sum(dr))
        patch = self.wire.empty(D, dev)
        if D:
            K.gather_wire(pl.req_recv, self.m.table.state, self.wire, patch, threads=self.m.cfg.threads,
                          idx=e.didx[:D], run_off=pl.run_off, W=W)
        if W == 1:
            recv = patch
        else:
            recv = self.wire.empty(Dr, dev)
            _a2a(recv, patch, dr, ds, self.group)
            self.bytes_sent += self.wire.rb * self._to_others(ds)
        if e.work is not None:
            e.work.wait()   # the early rows have arrived (compute stream waits on the RCCL stream)
            e.work = e.rows_send = None
        if Dr:
            off = np.zeros(W + 1, dtype=np.int32)
            off[1:] = np.cumsum(dr)
            recv_off = torch.from_numpy(off).pin_memory().to(dev, non_blocking=True)
            K.patch_scatter(recv, Dr, W, recv_off, e.sc_start, e.gathered)
        return self.wire.views(e.gathered)

    def _early_cpu(self, pl: _ShardPlan, cur: _ShardPlan) -> _Early:
        """CPU (gloo) reference of the early row exchange with plain torch ops: gather and
        exchange all rows of ``pl`` now, flag the ones the step being computed (plan ``cur``)
        will update -- they are re-gathered and re-sent after that update (``_patch_cpu``).
        The clean rows' values are final already: only ``cur``'s apply writes the table
        until then.  ``_early_gpu`` is the same with dedicated kernels."""
        W = self.W
        part = pl.parts[0]
        R, U = pl.R, pl.U
        req = pl.req_recv[:R]
        flags = K.run_member(req, cur.req_recv, cur.run_off, cur.splits).bool()
        run_of = torch.repeat_interleave(torch.arange(W), torch.tensor(part.rc), output_size=R)
        didx = torch.nonzero(flags).flatten()
        starts = torch.tensor(np.concatenate([[0], np.cumsum(part.rc)[:-1]]).astype(np.int64))
        e = _Early()
        e.dirty_rows = req[didx]
        e.dtags = (didx - starts[run_of[didx]]).to(torch.int32)
        e.dsend = torch.bincount(run_of[didx], minlength=W)      # dirty rows per source rank
        e.dpos = torch.tensor(np.concatenate([[0], np.cumsum(part.sc)[:-1]]).astype(np.int64))  # sc starts
        rows_send = self.wire.empty(R, self.dev)
        K.gather_wire(req, self.m.table.state, self.wire, rows_send, threads=self.m.cfg.threads)
        if W == 1:
            e.gathered = rows_send
        else:
            e.gathered = self.wire.empty(U, self.dev)
            _a2a(e.gathered, rows_send, part.sc, part.rc, self.plan_group)
            self.bytes_sent += self.wire.rb * self._to_others(part.rc)
        return e

    def _tag_view(self, buf: torch.Tensor) -> torch.Tensor:
        """int32 view of the last pad word of every wire row (carries a patch row's tag)."""
        w = buf.view(torch.int32) if buf.dtype != torch.int32 else buf
        col = (self.Kp + 3) if self.wire.fp32 else (self.wire.vb // 4 + 3)
        return w[:, col]

    def _patch_cpu(self, pl: _ShardPlan) -> tuple[torch.Tensor, torch.Tensor]:
        """CPU reference of ``_patch_gpu``: after the previous step's update, re-gather the
        dirty rows (tagged with their index in their source's run), send them to their
        requesters and overwrite the early copies; returns the (v, w) views."""
        e, W = pl.early, self.W
        dsend = e.dsend
        if W == 1:
            drecv = dsend
        else:
            drecv = torch.empty_like(dsend)
            dist.all_to_all_single(drecv, dsend, group=self.cpu_group)
        ds, dr = dsend.tolist(), drecv.tolist()
        patch = self.wire.empty(len(e.dirty_rows), self.dev)
        K.gather_wire(e.dirty_rows, self.m.table.state, self.wire, patch, threads=self.m.cfg.threads)
        self._tag_view(patch).copy_(e.dtags)
        if W == 1:
            recv = patch
        else:
            recv = self.wire.empty(int(sum(dr)), self.dev)
            _a2a(recv, patch, dr, ds, self.group)
            self.bytes_sent += self.wire.rb * self._to_others(ds)
        if recv.shape[0]:
            base = torch.repeat_interleave(e.dpos, drecv)
            e.gathered.index_copy_(0, base + self._tag_view(recv).to(torch.int64), recv)
        return self.wire.views(e.gathered)

    def _split_ok(self, pl: _ShardPlan, dd) -> bool:
        return self.overlap_grads and len(pl.parts) == 1

    def _half_bounds(self, part: _Part) -> tuple[list[int], list[int], list[int], list[int]]:
        """Per owner q: start of my requests to q in unique order, and the size of their first half;
        per source s: start of s's run in my received requests, and the size of its first half
        (the sender's first half of a run of n rows is (n + 1) // 2 on both sides)."""
        sc, rc = part.sc, part.rc
        s_start = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.int64).tolist()
        r_start = np.concatenate([[0], np.cumsum(rc)[:-1]]).astype(np.int64).tolist()
        return s_start, [(n + 1) // 2 for n in sc], r_start, [(n + 1) // 2 for n in rc]

    def _split_plan(self, pl: _ShardPlan) -> None:
        """Once per plan (in its finish, off the step): the split backward's per-owner segment bounds
        (device int32 [2W + 1], staged on the finish stream) and, per piece, every peer's send / receive
        row ranges -- the step only wraps them in one all-to-all (P2P ops on CPU)."""
        part = pl.parts[0]
        s_start, s_half, r_start, r_half = self._half_bounds(part)
        pieces = []
        for piece in (0, 1):
            rng = []
            for q in range(self.W):
                a0 = s_start[q] + (0 if piece == 0 else s_half[q])
                a1 = s_start[q] + (s_half[q] if piece == 0 else part.sc[q])
                b0 = r_start[q] + (0 if piece == 0 else r_half[q])
                b1 = r_start[q] + (r_half[q] if piece == 0 else part.rc[q])
                rng.append((q, a0, a1, b0, b1))
            pieces.append(rng)
        pl.pieces = pieces
        if self.dev.type == "cuda":
            sb = []
            for q in range(self.W):
                sb += [s_start[q], s_start[q] + s_half[q]]
            sb.append(part.U)
            slot = self.slots[pl.slot]
            if getattr(slot, "sb_h", None) is None or slot.sb_h.numel() != len(sb):
                slot.sb_h = torch.empty(len(sb), dtype=torch.int32, pin_memory=True)
                slot.sb = torch.empty(len(sb), dtype=torch.int32, device=self.dev)
            slot.sb_h.numpy()[:] = sb  # (this slot's previous copy finished: its plan's step is over)
            slot.sb.copy_(slot.sb_h, non_blocking=True)
            pl.sb = slot.sb

    def _p2p_piece(self, pl: _ShardPlan, piece: int, grad_send: torch.Tensor, grad_recv: torch.Tensor):
        """Send every owner its rows of ``piece`` (0: first halves, 1: second halves) and receive
        the matching rows of every source into their place in ``grad_recv`` (rank-major runs).
        Returns the pending works."""
        if self.W == 1:
            return []  # (grad_recv is grad_send)
        if self.dev.type == "cuda":
            # one all-to-all over per-peer views (the own chunk included): a single C++ call issues the
            # RCCL group of sends / receives, where 2 (W - 1) Python P2P ops per piece cost host time
            # that grows with W
            ins = [grad_send[a0:a1] for _, a0, a1, _, _ in pl.pieces[piece]]
            outs = [grad_recv[b0:b1] for _, _, _, b0, b1 in pl.pieces[piece]]
            w = dist.all_to_all(outs, ins, group=self.group, async_op=True)
            return [w] if w is not None else []
        ops, me = [], self.ctx.rank
        for q, a0, a1, b0, b1 in pl.pieces[piece]:
            if q == me:
                if b1 > b0:
                    grad_recv[b0:b1].copy_(grad_send[a0:a1])
                continue
            if a1 > a0:
                ops.append(dist.P2POp(dist.isend, grad_send[a0:a1], q, group=self.group))
            if b1 > b0:
                ops.append(dist.P2POp(dist.irecv, grad_recv[b0:b1], q, group=self.group))
        if not ops:
            return []
        return [op.op(op.tensor, op.peer, group=op.group) for op in ops]  # (CPU / gloo)

    def _bwd_split_exchange(self, pl, part, dd, fo, src_v, src_w, gs, grad_recv, rv, rw, skw) -> list:
        """Backward in two pieces (every owner's first half of rows, then the second half) with
        the first piece's gradient rows sent while the second is reduced."""
        m, ws, cfg, Kp, wf = self.m, self.m.ws, self.m.cfg, self.Kp, self.wire
        if pl.pieces is None:  # (a plan finished before its split ranges existed)
            self._split_plan(pl)
        if self.W > 1:
            self.bytes_sent += 4 * wf.g_words * self._to_others(part.sc)
        kw = dict(mode=K.BWD_EMIT, src_v=src_v, src_w=src_w, grad_out=gs, reg_v=rv, reg_w=rw,
                  partial=ws.bwd_partial, threads=cfg.threads, grad_bf16=wf.grad_bf16, **skw)
        if self.dev.type != "cuda":  # CPU reference: one backward, the exchange still in two pieces
            K.fm_backward(dd, fo.dpred, fo.r1, Kp, **kw)
            return self._p2p_piece(pl, 0, gs, grad_recv) + self._p2p_piece(pl, 1, gs, grad_recv)
        K.fm_backward(dd, fo.dpred, fo.r1, Kp, seg_bounds=pl.sb, piece=0, **kw)
        works = self._p2p_piece(pl, 0, gs, grad_recv)
        K.fm_backward(dd, fo.dpred, fo.r1, Kp, seg_bounds=pl.sb, piece=1, **kw)
        return works + self._p2p_piece(pl, 1, gs, grad_recv)

    def _check_splits(self, part: _Part) -> None:
        """FM_DEBUG_CHECKS=1: the split lists of every rank must form a consistent W x W
        exchange (what rank s sends to r is what r expects from s) and cover all unique ids."""
        mats = [None] * self.W
        dist.all_gather_object(mats, (part.sc, part.rc), group=self.cpu_group)
        for r in range(self.W):
            for q in range(self.W):
                if mats[q][0][r] != mats[r][1][q]:
                    raise RuntimeError(f"a2a split mismatch: rank {q} sends {mats[q][0][r]} ids to rank {r}, "
                                       f"which expects {mats[r][1][q]}")
        dd = part.dd
        u = int(dd.num_unique.item())
        if u != part.U:
            raise RuntimeError(f"owner counts cover {part.U} ids, dedup found {u}")
        if part.U and int(dd.uniq[part.U - 1].item()) >= self.W * self.Rps:
            raise RuntimeError("sharded key out of range")

    def _drop_pending(self) -> None:
        """The caller broke the batch order it promised (``next_batch`` / ``next2``): the pending
        plans are for batches that are not coming next -- drop them (their slots free again; every
        rank drops the same plans, since the call sequence is the same on all ranks)."""
        for p in self.pending:
            e = getattr(p, "early", None)
            if e is not None and getattr(e, "work", None) is not None:
                e.work.wait()
                e.work = None
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)  # (rare path: nothing in flight may still use the slots)
        self.pending = []

    def _take_plan(self, b: Batch, train: bool) -> _ShardPlan:
        if train and self.pending and self.pending[0].b is not b:
            self._drop_pending()
        pl = self.pending[0] if (self.pending and train) else None
        if pl is not None and pl.b is b and (len(pl.parts) > 1) == (self.nparts > 1 and b.B >= 2 * self.nparts):
            self.pending.pop(0)
            self._plan_finish(pl)
        else:  # (evaluation: the pending training plans stay pending)
            pl = self._plan(b, train, early=False)
        if pl.ready is not None:
            main = torch.cuda.current_stream(self.dev)
            main.wait_event(pl.ready)
            pl.req_recv.record_stream(main)  # allocated on the side stream, read on main
            for part in pl.parts:
                if part.b is not b:
                    part.b.offsets.record_stream(main)
            if pl.early is not None:
                e = pl.early
                for t in (e.gathered, e.didx, e.sc_start):
                    if t is not None:
                        t.record_stream(main)
        return pl

    def _gather_part(self, pl: _ShardPlan, part: _Part, async_op: bool):
        """Owner gather of the rows part ``part`` requested + a2a back.

        Returns (buffer, work): the U wire rows in unique order arrive in ``buffer``
        once ``work`` (None: already there) is waited for."""
        rows_send = self.wire.empty(part.R, self.dev)
        K.gather_wire(pl.req_recv[part.r0: part.r0 + part.R], self.m.table.state, self.wire, rows_send,
                      threads=self.m.cfg.threads, skip=pl.self_r)
        if self.W == 1:
            return rows_send, None
        gathered = self.wire.empty(part.U, self.dev)
        work = dist.all_to_all_single(gathered, rows_send, part.sc, part.rc, group=self.group, async_op=async_op)
        self.bytes_sent += self.wire.rb * self._to_others(part.rc)
        return gathered, work

    def train_step(self, b: Batch, next_batch: Batch | None = None, next2: Batch | None = None):
        """One step on ``b``.  ``next_batch`` / ``next2``: the batches of the next two calls.

        Depth-1 (``next_batch`` only): the plan of the next batch is built at the end of this
        step (and, with early rows, its early exchange right after).  Depth-2 (both): the plan
        of ``next2`` is built at the end of this step, and at the start of this step the early
        row exchange of the next batch (planned during the previous step) is launched, so the
        whole table-independent half of a step and its row exchange have a full step of slack."""
        from ..models.fm import StepOut

        if self.dev.type == "cuda":
            self._main = torch.cuda.current_stream(self.dev)
        if self.staleness:
            return self._train_step_stale(b, next_batch, next2)
        if self.local_w1:  # (see __init__)
            if next_batch is not None or self.m._lpending is not None:
                return self.m._local_lookahead_step(b, next_batch, next2)
            return self.m._local_train_step(b)
        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        gpu = self.dev.type == "cuda"
        build = next2 if next2 is not None else next_batch
        nb_ready = None
        if build is not None and gpu and getattr(build, "ready", None) is None:
            nb_ready = torch.cuda.Event()  # the batch's producers: all work enqueued before this step
            nb_ready.record(self._main)
        if gpu:
            self.step_start = torch.cuda.Event()  # after the previous step's apply (early gathers wait on it)
            self.step_start.record(self._main)
        with roctx_range("plan"):
            pl = self._take_plan(b, True)
        self.cur_plan = pl
        wf = self.wire
        # every part's rows are gathered first and their all-to-alls queued on RCCL's stream
        # (async): part k+1's rows travel while part k computes
        with roctx_range("gather+a2a_rows"):
            if pl.early is not None:
                rows = [(None, None)]
                early_views = self._patch(pl)
                self.early_steps += 1
            else:
                rows = [self._gather_part(pl, part, async_op=True) for part in pl.parts]
        grad_send = wf.empty_grads(max(pl.U, 1), self.dev)
        grad_recv = grad_send if self.W == 1 else wf.empty_grads(max(pl.R, 1), self.dev)
        gworks = []
        loss = None
        rv, rw = m.reg_coeffs
        gscale = m.grad_scale(b.B)
        # (one stochastic-rounding tick per step, shared by the in-place self-row updates of the
        # backward and the owner's apply: the same row gets the same bits either way)
        sr = m.sr_tick()
        srows, skw = None, {}
        if pl.self_u is not None:
            srows = K.SelfRows(pl.self_u[0], pl.self_u[1], self.ctx.rank * self.Rps, pl.parts[0].dd.uniq,
                               m.table.state, pl.self_excl)
            skw = dict(self_rows=srows, opt=cfg.opt, sr_counter=sr)
        # one part: the loss reduction is enqueued after the backward, as in the local step
        one_part = len(pl.parts) == 1
        for part, (buf, work) in zip(pl.parts, rows):
            sb, dd, e0 = part.b, part.dd, part.e0
            if work is not None:
                work.wait()               # the compute stream waits for this part's rows
            src_v, src_w = wf.views(buf) if buf is not None else early_views
            gs = grad_send[part.u0: part.u0 + part.U]
            with roctx_range("fwd"):
                fo = K.fm_forward(sb.offsets, part.keys if part.seg is not None else dd.inv[: sb.nnz], sb.vals,
                                  src_v, src_w, Kp, labels=sb.labels,
                                  weights=sb.weights, loss=cfg.loss_type, grad_scale=gscale, want_r1=True,
                                  pred=ws.pred[e0: e0 + sb.B], r1=ws.r1[e0: e0 + sb.B],
                                  dpred=ws.dpred[e0: e0 + sb.B], partial=ws.fwd_partial, threads=cfg.threads,
                                  bias=m.gbias, self_rows=srows, seg_lookup=part.seg, defer_loss=one_part)
            if not one_part:  # (the parts share the loss partials: each part's sum before the next)
                loss = fo.loss_sum if loss is None else loss + fo.loss_sum
            if self._split_ok(pl, dd):
                with roctx_range("bwd_split+grads"):
                    gworks += self._bwd_split_exchange(pl, part, dd, fo, src_v, src_w, gs, grad_recv, rv, rw, skw)
                continue
            with roctx_range("bwd"):
                K.fm_backward(dd, fo.dpred, fo.r1, Kp, mode=K.BWD_EMIT, src_v=src_v, src_w=src_w, grad_out=gs,
                              reg_v=rv, reg_w=rw, partial=ws.bwd_partial, threads=cfg.threads,
                              grad_bf16=wf.grad_bf16, **skw)
            if self.W > 1:
                with roctx_range("a2a_grads"):
                    gworks.append(dist.all_to_all_single(grad_recv[part.r0: part.r0 + part.R], gs, part.rc, part.sc,
                                                         group=self.group, async_op=True))
                    self.bytes_sent += 4 * wf.g_words * self._to_others(part.sc)
        m.bias_step(ws.dpred[: b.B])
        if one_part:
            loss = fo.finish_loss()
        for w in gworks:
            w.wait()
        with roctx_range("apply"):
            if not (srows is not None and self.W == 1):  # (world 1: updated in place)
                K.apply_runs(pl.req_recv, pl.run_off, pl.splits, grad_recv, m.table.state, cfg.opt, Kp,
                             match=pl.match, threads=cfg.threads,
                             ws=self.slots[pl.slot].ensure2(pl.R, self.dev) if not gpu else None,
                             grad_bf16=wf.grad_bf16, sr_counter=sr, self_run=self.ctx.rank if srows else -1,
                             self_excl=pl.self_excl)
        if gpu:
            done = torch.cuda.Event()
            done.record(self._main)
            self.slots[pl.slot].done = done
        if self.pending and next_batch is not None and self.pending[0].b is next_batch:
            # Finish the next batch's plan only now, with this whole step already enqueued: the
            # host's wait for its owner counts (dedup on the plan stream, started one step ago)
            # then overlaps this step's GPU work instead of holding back the step's launches
            # (at the start of the step it left the compute stream idle ~270 us per step at
            # world 1: profiles/shard_w1_r1s3/timeline_early_split_off.txt).  Its early row
            # exchange gathers against the table as of this step's start (step_start) and is
            # patched after this step's update.
            nxt_pl = self.pending[0]
            with roctx_range("plan_finish_next"):
                self._plan_finish(nxt_pl)
            if nxt_pl.early is None and self._early_ok(nxt_pl, pl):
                with roctx_range("early_rows_next"):
                    self._early_ahead(nxt_pl, pl)
        if next2 is not None and not any(p.b is next2 for p in self.pending):
            if not any(p.b is next_batch for p in self.pending) and next_batch is not None:
                with roctx_range("plan_next"):  # (first depth-2 step: the next batch has no plan yet)
                    self.pending.append(self._plan(next_batch, True, nb_ready, early=True))
            with roctx_range("plan_next2"):  # started now, finished at the start of the next step
                self.pending.append(self._plan_start(next2, True, nb_ready))
        elif next2 is None and next_batch is not None and not any(p.b is next_batch for p in self.pending):
            with roctx_range("plan_next"):
                if self.prefetch_depth1:  # built in full now, with its early row exchange
                    self.pending.append(self._plan(next_batch, True, nb_ready, early=True))
                else:  # started now, finished when the next step takes it
                    self.pending.append(self._plan_start(next_batch, True, nb_ready))
        return StepOut(loss, b.B)

    @torch.no_grad()
    def forward(self, b: Batch, *, loss: str = "none", want_reg: bool = False) -> K.FwdOut:
        self.flush()  # (staleness: evaluate the table with every update applied)
        self.m.ws.ensure(b.B, b.nnz)
        pl = self._take_plan(b, False)
        part = pl.parts[0]
        buf, work = self._gather_part(pl, part, async_op=False)
        src_v, src_w = self.wire.views(buf)
        seg = getattr(part, "seg", None)  # (eval plans keep the inverse map: train=False)
        out = K.fm_forward(b.offsets, part.keys if seg is not None else part.dd.inv[: b.nnz], b.vals, src_v, src_w,
                           self.Kp, labels=b.labels, weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False,
                           want_reg=want_reg, threads=self.m.cfg.threads, bias=self.m.gbias, seg_lookup=seg)
        if self.dev.type == "cuda":
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.dev))
            self.slots[pl.slot].done = done
        return out


class DPExchange(_Base):
    """Replicated table; sparse all-gather of (ids, gradient rows)."""

    def _local_grads(self, b: Batch):
        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        rows = m._rows32(b)
        ex = K.csr_rows(b.offsets, out=ws.dd.ex_of_occ[: b.nnz], nnz=b.nnz)
        fo = K.fm_forward(b.offsets, rows, b.vals, m.table.v, m.table.w, Kp, labels=b.labels, weights=b.weights,
                          loss=cfg.loss_type, grad_scale=m.grad_scale(b.B), want_r1=True, pred=ws.pred[: b.B],
                          r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial, threads=cfg.threads,
                          bias=m.gbias, max_feats=b.max_feats)
        m.bias_step(fo.dpred)
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
        # (ring all-gather: each rank forwards W - 1 chunks of its padded size)
        self.bytes_sent += (self.W - 1) * (ids_pad.numel() * 4 + g_pad.numel() * 4 + 8)
        ids_cat = torch.cat([ids_all[r][: sizes[r]] for r in range(self.W)])
        g_cat = torch.cat([g_all[r][: sizes[r]] for r in range(self.W)])
        n = ids_cat.numel()
        dd2 = K.dedup(ids_cat, ws=self._dd2(n), key_bits=bits_for(self.m.table.rows), want_perm=True)
        K.apply_rows(dd2, g_cat, self.m.table.state, self.m.cfg.opt, self.Kp, threads=self.m.cfg.threads,
                     sr_counter=self.m.sr_tick())
        return StepOut(fo.loss_sum, b.B)

    @torch.no_grad()
    def forward(self, b: Batch, *, loss: str = "none", want_reg: bool = False) -> K.FwdOut:
        t = self.m.table
        return K.fm_forward(b.offsets, b.ids.to(torch.int32), b.vals, t.v, t.w, self.Kp, labels=b.labels,
                            weights=b.weights, loss=loss, grad_scale=1.0, want_r1=False, want_reg=want_reg,
                            threads=self.m.cfg.threads, bias=self.m.gbias, max_feats=b.max_feats)


def dp_dense_blocks(world: int) -> int:
    """Row blocks of the dp_dense step's pipeline (FM_DP_BLOCKS; default 4 at world > 1, 1 alone)."""
    v = os.environ.get("FM_DP_BLOCKS")
    return max(1, int(v)) if v else (4 if world > 1 else 1)


class DPDenseExchange(DPExchange):
    """Replicated table; dense gradient buffer reduce-scattered over the ranks, each rank updating
    its own rows, the updated rows all-gathered (small vocabularies, BASELINE config 3).

    Ownership: the replica's V rows form P blocks of Vb = V / P rows (FM_DP_BLOCKS, ``dp_dense_blocks``);
    block p's rows [p Vb + r Sb, p Vb + (r+1) Sb), Sb = Vb / W, belong to rank r (V is padded to a
    multiple of W P, FMTable ``rows_multiple``), so every block's reduce-scatter / all-gather is
    one in-place collective over a contiguous range.

    GPU step (no host synchronisation, lookahead dedup as in the local step), pipelined over the
    blocks -- each collective is issued asynchronously on the communicator's stream right after its
    inputs are enqueued, so it runs beside the compute stream's next piece:
      dedup of this batch (side stream, done during the previous step) -> forward on the replica
      -> per block p: backward piece p in EMIT_TABLE mode (the segments whose keys fall in block p:
      each unique row's [g_v | g_w | 1] scattered into the persistent dense buffer ``G`` [V, Kp+4],
      the touch word marking it) -> reduce-scatter of block p of ``G`` (RS(p) runs while piece
      p+1 is reduced; ``comm_dtype = bf16`` halves the bytes)
      -> per block p: wait RS(p) -> ``dense_apply`` of the own rows of block p (the optimizer's
      read-modify-write split W ways, every touched own row zeroed in ``G``) -> all-gather of
      block p's [v] and [w] rows (AG(p) runs while block p+1 is applied)
      -> this rank's scattered rows of the OTHER ranks' ranges are zeroed (``zero_listed_rows`` over
      the dedup's unique rows), so ``G`` is never cleared wholesale -> the compute stream waits
      for the all-gathers: identical replicas.  The next batch's dedup (side stream) runs beside.
    Bytes per rank and step: (W-1)/W of the buffer (reduce-scatter) + (W-1)/W of the parameter
    rows (all-gather), the same as the all-reduce it replaces, but the apply work no longer
    repeats on every rank and the optimizer state is only ever touched by its rows' owner
    (``sync_state`` all-gathers it for checkpoints).  What cannot overlap in a synchronous step:
    the forward (it reads every block's updated rows) and the last block's collectives
    (``tools/comm_model.py``).  The CPU (gloo) path follows the same ownership with plain torch
    ops (gloo has no reduce-scatter: the all-reduced buffer's rows are the same sums)."""

    supports_lookahead = True

    def __init__(self, model):
        super().__init__(model)
        V = model.table.rows
        self.P = dp_dense_blocks(self.W)
        if V % (self.W * self.P):
            raise ValueError("dp_dense: the replicated table's rows must be a multiple of world size x blocks")
        self.Vb = V // self.P
        self.Sb = self.Vb // self.W
        self.dense = torch.zeros((V, self.gs), dtype=torch.float32, device=self.dev)
        self.arange = torch.arange(V + 1, dtype=torch.int32, device=self.dev)
        self.wire16 = (torch.empty((V, self.gs), dtype=torch.bfloat16, device=self.dev)
                       if self.dev.type == "cuda" and model.cfg.comm_dtype == "bf16" else None)
        self.bounds = torch.zeros(self.P + 2, dtype=torch.int32, device=self.dev)
        self.local_w1 = (self.W == 1 and self.dev.type == "cuda" and os.environ.get("FM_DP_W1_LOCAL", "1") != "0")

    def close(self) -> None:
        self.dense = self.wire16 = None
        super().close()

    def own_range(self, p: int) -> tuple[int, int]:
        """Rows [a, b) of block p owned by this rank."""
        a = p * self.Vb + self.ctx.rank * self.Sb
        return a, a + self.Sb

    def _param_tensors(self) -> list[torch.Tensor]:
        """The replica's parameter tensors, rows first (all-gathered after the sharded apply)."""
        t = self.m.table
        v = t.v.view(torch.uint8) if t.fp8 else t.v
        return [v, t.wx if t.fp8 else t.w]

    def _state_tensors(self) -> list[torch.Tensor]:
        t = self.m.table
        return [x for x in (t.s0v, t.s0w, t.s1v, t.s1w) if x is not None]

    def _all_gather_block(self, tensors: list[torch.Tensor], p: int, async_op: bool = False) -> list:
        """Every rank's own rows of block p of each tensor to every rank, in place."""
        if self.W == 1:
            return []
        a, b = self.own_range(p)
        blk = slice(p * self.Vb, (p + 1) * self.Vb)
        works = []
        for t in tensors:
            if self.dev.type == "cuda":
                w = dist.all_gather_into_tensor(t[blk], t[a:b], group=self.group, async_op=async_op)
                if w is not None:
                    works.append(w)
            else:
                parts = [torch.empty_like(t[a:b]) for _ in range(self.W)]
                dist.all_gather(parts, t[a:b].contiguous(), group=self.group)
                t[blk].copy_(torch.cat(parts))
            self.bytes_sent += (self.W - 1) * t[a:b].numel() * t.element_size()
        return works

    def _all_gather_rows(self, tensors: list[torch.Tensor]) -> None:
        for p in range(self.P):
            self._all_gather_block(tensors, p)

    def sync_state(self) -> None:
        """All-gather the optimizer state (each rank's apply only updates its own rows' state):
        after this every replica holds the full state (checkpoints, re-sharding)."""
        if self.dev.type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()
        self._all_gather_rows(self._state_tensors())

    def _block_bounds(self, dd) -> torch.Tensor:
        """int32 [P + 2] device: first segment of each block (keys ascending), U twice at the end."""
        cnt = K.owner_counts(dd, self.Vb, self.P)
        self.bounds[1: self.P + 1].copy_(torch.cumsum(cnt, 0))
        self.bounds[self.P + 1: self.P + 2].copy_(self.bounds[self.P: self.P + 1])
        return self.bounds

    def _reduce_scatter_block(self, p: int):
        a, b = self.own_range(p)
        blk = slice(p * self.Vb, (p + 1) * self.Vb)
        if self.wire16 is not None:
            self.wire16[blk].copy_(self.dense[blk])
            w = dist.reduce_scatter_tensor(self.wire16[a:b], self.wire16[blk], group=self.group, async_op=True)
            self.bytes_sent += (self.W - 1) * self.Sb * self.gs * 2
        else:
            w = dist.reduce_scatter_tensor(self.dense[a:b], self.dense[blk], group=self.group, async_op=True)
            self.bytes_sent += (self.W - 1) * self.Sb * self.gs * 4
        return w

    def train_step(self, b: Batch, next_batch: Batch | None = None, next2: Batch | None = None):
        from ..models.fm import StepOut

        if self.dev.type != "cuda":
            return self._train_step_reference(b)
        if self.local_w1:
            # world 1: the replica is the whole table and this rank owns every row, so the step is the
            # local step (fused backward + in-place update of the touched rows only) -- the dense
            # buffer, its scan of all V rows by dense_apply (132 us of 0.72 ms at V = 1M) and the
            # zeroing are for the exchange (profiles/r5/dp_dense_w1.txt; FM_DP_W1_LOCAL=0: dense path)
            if next_batch is not None or self.m._lpending is not None:
                return self.m._local_lookahead_step(b, next_batch, next2)
            return self.m._local_train_step(b)
        m, ws, cfg, Kp = self.m, self.m.ws, self.m.cfg, self.Kp
        main = torch.cuda.current_stream(self.dev)
        nb_ready = None
        if next_batch is not None and getattr(next_batch, "ready", None) is None:
            nb_ready = torch.cuda.Event()
            nb_ready.record(main)
        pl = m._lpending
        if pl is not None and pl.b is b:
            m._lpending, m._lpending2 = m._lpending2, None
        else:
            m._lpending = m._lpending2 = None
            pl = m._local_plan(b)
        main.wait_event(pl.ready)
        with roctx_range("fwd"):
            fo = K.fm_forward(b.offsets, pl.rows, b.vals, m.table.v, m.table.w, Kp, labels=b.labels,
                              weights=b.weights, loss=cfg.loss_type, grad_scale=m.grad_scale(b.B), want_r1=True,
                              pred=ws.pred[: b.B], r1=ws.r1[: b.B], dpred=ws.dpred[: b.B], partial=ws.fwd_partial,
                              bias=m.gbias, max_feats=b.max_feats)
            m.bias_step(fo.dpred)
        rv, rw = m.reg_coeffs
        # backward pieces by key block, each block's reduce-scatter issued behind its piece
        pieces = self.W > 1 and self.P > 1
        bounds = self._block_bounds(pl.dd) if pieces else None
        rs = []
        with roctx_range("bwd_scatter+reduce_scatter"):
            for p in range(self.P if pieces else 1):
                K.fm_backward(pl.dd, fo.dpred, fo.r1, Kp, mode=K.BWD_EMIT_TABLE, table=m.table.state,
                              grad_out=self.dense, reg_v=rv, reg_w=rw, partial=ws.bwd_partial,
                              piece=0 if pieces else -1, seg_bounds=bounds[p: p + 3] if pieces else None)
                if pieces:
                    rs.append(self._reduce_scatter_block(p))
            if self.W > 1 and not pieces:
                rs = [self._reduce_scatter_block(p) for p in range(self.P)]
        # the next batches' dedup (side stream) overlaps the collectives, the apply and -- depth 2,
        # like the local step -- the next step's forward / backward
        # (this step's slot has no done event yet -- the apply and zero_listed_rows below still read
        # its plan -- so the new plans avoid it)
        if next_batch is not None and (m._lpending is None or m._lpending.b is not next_batch):
            m._lpending = m._local_plan(next_batch, nb_ready, avoid=pl.slot)
            m._lpending2 = None
        if (next2 is not None and m._lpending is not None and m._lpending2 is None
                and os.environ.get("FM_LOCAL_DEPTH2", "1") != "0"):
            if getattr(next2, "ready", None) is None and nb_ready is None:
                nb_ready = torch.cuda.Event()
                nb_ready.record(main)
            m._lpending2 = m._local_plan(next2, nb_ready, avoid=pl.slot)
        ag = []
        sr = m.sr_tick()
        with roctx_range("apply+all_gather"):
            for p in range(self.P):
                a, e = self.own_range(p)
                if self.W > 1:
                    rs[p].wait()  # (the compute stream waits for the communicator's stream)
                    if self.wire16 is not None:
                        self.dense[a:e].copy_(self.wire16[a:e])
                K.dense_apply(self.dense[a:e], m.table.state, cfg.opt, Kp, row0=a, rows=self.Sb, sr_counter=sr)
                ag += self._all_gather_block(self._param_tensors(), p, async_op=True)
        if self.W > 1:
            # this rank's contributions to the other ranks' rows (its own touched rows were zeroed
            # by the apply; re-zeroing them is harmless); every reduce-scatter has been waited for
            K.zero_listed_rows(self.dense, pl.dd.uniq, pl.dd.counts[:1], pl.dd.n)
            for w in ag:
                w.wait()
        done = torch.cuda.Event()
        done.record(main)
        m._lslots[pl.slot].done = done
        return StepOut(fo.loss_sum, b.B)

    def _train_step_reference(self, b: Batch):
        from ..models.fm import StepOut

        fo, uniq, grad = self._local_grads(b)
        dense = self.dense
        dense.zero_()
        idx = uniq.to(torch.int64)
        dense.index_copy_(0, idx, grad)
        dense[idx, self.Kp + 1] = 1.0  # touch counter travels in a pad column
        if self.W > 1:
            dist.all_reduce(dense, group=self.group)
            self.bytes_sent += 2 * (self.W - 1) * dense.numel() * 4 // self.W
        sr = self.m.sr_tick()
        for p in range(self.P):
            r0, r1 = self.own_range(p)
            own = dense[r0:r1]
            touched = torch.nonzero(own[:, self.Kp + 1] > 0).flatten().to(torch.int32)
            T = touched.numel()
            dd = K.DedupOut(n=T, uniq=touched + r0, perm=touched, seg_start=self.arange[: T + 1],
                            num_unique=torch.tensor([T], dtype=torch.int32, device=self.dev), U_host=T)
            K.apply_rows(dd, own, self.m.table.state, self.m.cfg.opt, self.Kp, threads=self.m.cfg.threads,
                         sr_counter=sr)
        self._all_gather_rows(self._param_tensors())
        return StepOut(fo.loss_sum, b.B)
