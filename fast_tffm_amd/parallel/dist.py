"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

Reference: TF gRPC cluster (``--dist JOB_NAME TASK_INDEX PS_HOSTS WORKER_HOSTS``
-> ClusterSpec + tf.train.Server, run_tffm.py:169-195), parameter servers that
block in ``server.join()`` and a worker start barrier polling a counter
variable every 0.2 s (run_tffm.py:207-226).

Here every rank is a worker that owns a shard of the table in its own HBM, so
there are no PS processes.  Rank/world come from torchrun's environment
(RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT), or from ``--dist``
(worker i of the WORKER_HOSTS list; the first worker host is the rendezvous).
The backend is "nccl" (= RCCL on ROCm) for GPU tensors and "gloo" on CPU.
"""

from __future__ import annotations

import datetime
import os
import weakref
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str
    group: object = None          # main process group (RCCL or gloo)
    cpu_group: object = None      # gloo side group for host-side barriers/objects

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def all_reduce_scalar(self, x: float, op: str = "sum") -> float:
        if self.world == 1:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        return float(t.item())


_CTX: DistContext | None = None
# objects holding communicators, streams or captured graphs (models / exchanges): closed, in
# creation order, before the process groups are destroyed
_LIVE: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()
_LIVE_SEQ = 0


def register_closeable(obj) -> None:
    """Track ``obj`` (with a ``close()`` method) so that ``shutdown()`` releases it first."""
    global _LIVE_SEQ
    _LIVE_SEQ += 1
    _LIVE[_LIVE_SEQ] = obj


def parse_dist_args(dist_args: list[str] | None) -> dict:
    """Map the reference's ``--dist JOB TASK PS_HOSTS WORKER_HOSTS`` onto rank/world/master."""
    if not dist_args:
        return {}
    job, task, _ps_hosts, worker_hosts = dist_args
    workers = [h for h in worker_hosts.split(",") if h]
    if job == "ps":
        return {"role": "ps"}
    if job != "worker":
        raise ValueError(f"--dist JOB_NAME must be 'ps' or 'worker', got {job!r}")
    host, _, port = workers[0].rpartition(":")
    return {"role": "worker", "rank": int(task), "world": len(workers), "master_addr": host or "127.0.0.1",
            "master_port": int(port) if port else 29500}


MIN_HW_QUEUES = 8
# GPU_MAX_HW_QUEUES as it stood when HIP initialised in this process (None: not known yet).
# HIP reads the variable once, at its first device call; later edits of the environment change
# nothing, so code that picks a stream layout by the queue count reads this, not the env.
_HWQ_IN_FORCE: int | None = None


def _env_hw_queues() -> int:
    return int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)


def ensure_hw_queues(n: int = MIN_HW_QUEUES) -> int:
    """Give this process >= ``n`` HIP hardware queues (GPU_MAX_HW_QUEUES, default 4): HIP maps
    streams round-robin onto them, and streams that share a queue execute in submission order.
    The multi-rank step keeps the compute, plan / lookahead and dense streams plus one RCCL
    stream per communicator busy at once; on shared queues they serialise (sharded step 1.43 ->
    1.18 ms measured with 8), and two communicators' collective kernels queued in opposite
    orders on two ranks could wait on each other.  Only effective before HIP initialises (the
    first device call): once it has, the environment is left alone, a warning is printed when
    the count in force is below ``n``, and the count in force is returned (``hw_queues()``)."""
    if _cuda_initialized():
        cur = hw_queues()
        if cur < n:
            import sys

            print(f"[fast_tffm_amd] warning: HIP already initialised with GPU_MAX_HW_QUEUES={cur} (< {n}); "
                  "multi-stream steps share hardware queues (single-communicator mode)", file=sys.stderr)
        return cur
    cur = _env_hw_queues()
    if cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)
        cur = n
    return cur


def _cuda_initialized() -> bool:
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001
        return False


def hw_queues() -> int:
    """Hardware queues of this process: the value HIP initialised with when known (recorded at
    the first call after initialisation), else the environment's current value."""
    global _HWQ_IN_FORCE
    if _HWQ_IN_FORCE is not None:
        return _HWQ_IN_FORCE
    cur = _env_hw_queues()
    if _cuda_initialized():
        _HWQ_IN_FORCE = cur   # (first look after HIP started: the environment has not moved since)
    return cur


def init_distributed(*, backend: str | None = None, rank: int | None = None, world: int | None = None,
                     master_addr: str | None = None, master_port: int | None = None,
                     device: str | None = None, timeout_s: float = 1800.0,
                     force_pg: bool = False) -> DistContext:
    """Initialise (or return) the process group for this process.

    ``force_pg`` creates a process group even at world size 1 (exercises the
    RCCL code paths on a single GPU).
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    world = int(world if world is not None else env_world)
    if world > 1 or force_pg:
        ensure_hw_queues()  # (before torch.cuda.is_available() below initialises HIP)
    rank = int(rank if rank is not None else os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", rank if world > 1 else 0))
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if use_gpu:
        n = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(n, 1))
        torch.cuda.set_device(dev)
        hw_queues()  # record the queue count HIP started with
    else:
        dev = torch.device("cpu")
    backend = backend or ("nccl" if use_gpu else "gloo")
    group = cpu_group = None
    if world > 1 or force_pg:
        if master_addr is not None:
            os.environ["MASTER_ADDR"] = master_addr
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if master_port is not None:
            os.environ["MASTER_PORT"] = str(master_port)
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")  # hang -> error, not a stuck job
        if not dist.is_initialized():
            timeout = datetime.timedelta(seconds=timeout_s)
            # torchrun --max-restarts re-runs every rank against the SAME rendezvous store;
            # keys of the failed attempt (e.g. the address of a sub-group's rank 0) would be
            # read back by the new processes, so each attempt gets its own key prefix
            store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world, timeout=timeout))
            attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
            store = dist.PrefixStore(f"fm_attempt_{attempt}", store)
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=timeout, store=store)
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        group = dist.group.WORLD
        cpu_group = dist.new_group(backend="gloo") if backend == "nccl" else group
    _CTX = DistContext(rank=rank, world=world, local_rank=local_rank, device=dev, backend=backend, group=group,
                       cpu_group=cpu_group)
    return _CTX


def local_context(device: str | torch.device = "cpu") -> DistContext:
    dev = torch.device(device)
    return DistContext(rank=0, world=1, local_rank=0, device=dev, backend="none")


def shutdown() -> None:
    """Close every live model / exchange (their communicators, streams and hipGraphs are
    released in a fixed order while the process groups still exist), then destroy the
    groups.  Nothing is left for the garbage collector to finalise after the destroy."""
    global _CTX
    for key in sorted(list(_LIVE.keys())):
        obj = _LIVE.get(key)
        if obj is not None:
            obj.close()
    _LIVE.clear()
    if dist.is_available() and dist.is_initialized():
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        dist.destroy_process_group()
    _CTX = None


def current() -> DistContext | None:
    return _CTX
