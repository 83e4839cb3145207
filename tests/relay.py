"""Asynchronous host relay of torch.distributed collectives on GPU tensors (tests only).

RCCL refuses two ranks on one device, so multi-rank GPU tests run gloo process groups and route
every collective the executors issue on CUDA tensors through this relay.  It reproduces the
stream semantics of ProcessGroupNCCL instead of completing on return:

* the collective is ordered after everything enqueued so far on the caller's current stream
  (its comm stream -- one per process group, like an RCCL communicator's -- waits on it);
* its result lands LATE: the comm stream spins (``torch.cuda._sleep``) before the pinned-host
  -> device copy into the output;
* ``async_op=True`` returns a Work whose ``wait()`` makes the current stream wait on the comm
  stream (no host block); ``async_op=False`` makes the current stream wait before returning;
* the inputs must stay untouched until the collective has finished: after the spin, the comm
  stream compares every input with its value at call time and counts mismatches in
  ``violations()`` (a missing stream wait / record_stream on a reused send buffer).

A missing ``work.wait()``, stream wait or event order in the executor then reads stale outputs
(results differ from the single-process reference) or counts a violation.  The data itself
moves over gloo on the host (pinned copies), so the exchange is exact.
"""

from __future__ import annotations

import torch
import torch.distributed as tdist

_STATE: dict = {}


class RelayWork:
    def __init__(self, ev: torch.cuda.Event):
        self.ev = ev

    def wait(self, timeout=None):
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self):
        return self.ev.query()

    def synchronize(self):
        self.ev.synchronize()


def violations() -> int:
    f = _STATE.get("flag")
    return 0 if f is None else int(f.item())


def _flag() -> torch.Tensor:
    # (created at the first collective: install() runs before the process group, and touching the
    # device there would start HIP before dist.ensure_hw_queues raised its queue count)
    if _STATE.get("flag") is None:
        _STATE["flag"] = torch.zeros(1, dtype=torch.int32, device="cuda")
    return _STATE["flag"]


def _comm_stream(group) -> torch.cuda.Stream:
    key = id(group) if group is not None else 0
    s = _STATE["streams"].get(key)
    if s is None:
        s = _STATE["streams"][key] = torch.cuda.Stream()
    return s


def _begin(inputs):
    """Device snapshots of the inputs (on the current stream) and their host copies."""
    cur = torch.cuda.current_stream()
    snaps = [t.clone() for t in inputs]
    cur.synchronize()
    return cur, snaps, [s.cpu() for s in snaps]


def _deliver(group, cur, inputs, snaps, outs, async_op):
    """On the group's comm stream, after the caller's work and a spin: check the inputs are
    unchanged, then copy every (device dst, host src) pair; the Work (or the wait) follows."""
    cs = _comm_stream(group)
    cs.wait_stream(cur)
    pinned = [(d, s.contiguous().pin_memory()) for d, s in outs]
    with torch.cuda.stream(cs):
        torch.cuda._sleep(_STATE["delay"])
        for t, s in zip(inputs, snaps):
            _flag().add_((t != s).any().to(torch.int32))
        for d, s in pinned:
            d.copy_(s.view(d.shape), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
    for t in list(inputs) + list(snaps) + [d for d, _ in outs]:
        t.record_stream(cs)
    w = RelayWork(ev)
    if async_op:
        return w
    w.wait()
    return None


def install(delay_cycles: int = 2_000_000) -> None:
    """Patch torch.distributed's GPU collectives used by the executors (idempotent)."""
    if _STATE:
        return
    real = dict(a2a=tdist.all_to_all_single, isend=tdist.isend, irecv=tdist.irecv,
                all_reduce=tdist.all_reduce, all_gather=tdist.all_gather,
                agit=tdist.all_gather_into_tensor, rst=tdist.reduce_scatter_tensor,
                bir=tdist.batch_isend_irecv, a2a_list=tdist.all_to_all)
    _STATE.update(streams={}, delay=int(delay_cycles), real=real, flag=None)

    def a2a(out, inp, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
        if not (out.is_cuda or inp.is_cuda):
            return real["a2a"](out, inp, output_split_sizes, input_split_sizes, group=group, async_op=async_op)
        cur, snaps, host = _begin([inp])
        o = torch.empty(out.shape, dtype=out.dtype)
        real["a2a"](o, host[0], output_split_sizes, input_split_sizes, group=group)
        return _deliver(group, cur, [inp], snaps, [(out, o)], async_op)

    def all_to_all(out_list, in_list, group=None, async_op=False):
        """List all-to-all (per-peer views) over gloo's all_to_all_single on the flattened chunks."""
        if not any(t.is_cuda for t in list(in_list) + list(out_list)):
            return real["a2a_list"](out_list, in_list, group=group, async_op=async_op)
        cur, snaps, host = _begin(list(in_list))
        in_splits = [h.numel() for h in host]
        out_splits = [o.numel() for o in out_list]
        flat = torch.cat([h.reshape(-1) for h in host]) if host else torch.empty(0)
        o = torch.empty(sum(out_splits), dtype=out_list[0].dtype)
        real["a2a"](o, flat, out_splits, in_splits, group=group)
        outs = [(d, part.view(d.shape)) for d, part in zip(out_list, o.split(out_splits))]
        return _deliver(group, cur, list(in_list), snaps, outs, async_op)

    def batch_isend_irecv(ops):
        sends = [op for op in ops if op.op in (tdist.isend, real["isend"])]
        recvs = [op for op in ops if op not in sends]
        cur, snaps, host = _begin([op.tensor for op in sends])
        works, outs = [], []
        for op, h in zip(sends, host):
            works.append(real["isend"](h, op.peer, group=op.group))
        for op in recvs:
            buf = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
            works.append(real["irecv"](buf, op.peer, group=op.group))
            outs.append((op.tensor, buf))
        for w in works:
            w.wait()
        group = ops[0].group if ops else None
        return [_deliver(group, cur, [op.tensor for op in sends], snaps, outs, True)]

    def _reduce(x, op, group):
        """gloo all-reduce of a host tensor (16-bit floats summed in fp32)."""
        if x.dtype in (torch.bfloat16, torch.float16):
            y = x.float()
            real["all_reduce"](y, op=op, group=group)
            return y.to(x.dtype)
        real["all_reduce"](x, op=op, group=group)
        return x

    def all_reduce(t, op=tdist.ReduceOp.SUM, group=None, async_op=False):
        if not t.is_cuda:
            return real["all_reduce"](t, op=op, group=group, async_op=async_op)
        cur, snaps, host = _begin([t])
        return _deliver(group, cur, [t], snaps, [(t, _reduce(host[0], op, group))], async_op)

    def all_gather(tensor_list, t, group=None, async_op=False):
        if not t.is_cuda:
            return real["all_gather"](tensor_list, t, group=group, async_op=async_op)
        cur, snaps, host = _begin([t])
        bufs = [torch.empty(x.shape, dtype=x.dtype) for x in tensor_list]
        real["all_gather"](bufs, host[0], group=group)
        return _deliver(group, cur, [t], snaps, list(zip(tensor_list, bufs)), async_op)

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        if not out.is_cuda:
            return real["agit"](out, inp, group=group, async_op=async_op)
        cur, snaps, host = _begin([inp])
        W = tdist.get_world_size(group)
        bufs = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(W)]
        real["all_gather"](bufs, host[0], group=group)
        return _deliver(group, cur, [inp], snaps, [(out, torch.cat(bufs).view(out.shape))], async_op)

    def reduce_scatter_tensor(out, inp, op=tdist.ReduceOp.SUM, group=None, async_op=False):
        if not out.is_cuda:
            return real["rst"](out, inp, op=op, group=group, async_op=async_op)
        cur, snaps, host = _begin([inp])
        full = _reduce(host[0].clone(), op, group)
        r = tdist.get_rank(group)
        n = out.numel()
        return _deliver(group, cur, [inp], snaps, [(out, full.reshape(-1)[r * n:(r + 1) * n])], async_op)

    import functools
    import time

    _STATE["t"] = 0.0

    def timed(fn):
        """Host seconds spent inside the relay (its staging, host syncs and gloo transfers): excluded
        when the executor's own host time is measured under the relay."""
        @functools.wraps(fn)
        def f(*a, **kw):
            t0 = time.perf_counter()
            try:
                return fn(*a, **kw)
            finally:
                _STATE["t"] += time.perf_counter() - t0
        return f

    tdist.all_to_all_single = timed(a2a)
    tdist.all_to_all = timed(all_to_all)
    tdist.batch_isend_irecv = timed(batch_isend_irecv)
    tdist.all_reduce = timed(all_reduce)
    tdist.all_gather = timed(all_gather)
    tdist.all_gather_into_tensor = timed(all_gather_into_tensor)
    tdist.reduce_scatter_tensor = timed(reduce_scatter_tensor)


def relay_seconds() -> float:
    """Host time spent inside relayed collectives so far."""
    return float(_STATE.get("t", 0.0))
