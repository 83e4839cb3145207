"""Row-sharded step at world W > 1 on ONE GPU, at bench scale, for kernel profiling.

RCCL refuses two ranks on one device, so (as in tests/test_dist_gpu_relay.py) the ranks talk
over gloo and the exchange's all-to-alls on GPU tensors are staged through host memory.  The
wall time is therefore meaningless (host copies, two ranks sharing one GPU); what this tool is
for is the per-kernel GPU time of the W > 1 path -- owner gathers, run-merge apply, dirty scan
and patch of the early row exchange, self rows, segment lookup -- under
``rocprofv3 --kernel-trace --stats -- python3 tools/relay_bench.py``.

usage: relay_bench.py [--world 2] [--steps 10] [--slots-per-gpu 62500000]
"""

from __future__ import annotations

import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


def _install_relay():
    import torch
    import torch.distributed as tdist

    real_a2a, real_isend, real_irecv = tdist.all_to_all_single, tdist.isend, tdist.irecv

    def a2a(out, inp, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
        if not (out.is_cuda or inp.is_cuda):
            return real_a2a(out, inp, output_split_sizes, input_split_sizes, group=group, async_op=async_op)
        o = torch.empty(out.shape, dtype=out.dtype)
        real_a2a(o, inp.cpu(), output_split_sizes, input_split_sizes, group=group)
        out.copy_(o)
        return _Done() if async_op else None

    def batch_isend_irecv(ops):
        works, recvs = [], []
        for op in ops:
            if op.op in (tdist.isend, real_isend):
                works.append(real_isend(op.tensor.cpu(), op.peer, group=op.group))
            else:
                buf = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
                works.append(real_irecv(buf, op.peer, group=op.group))
                recvs.append((op.tensor, buf))
        for w in works:
            w.wait()
        for t, buf in recvs:
            t.copy_(buf)
        return [_Done()]

    tdist.all_to_all_single = a2a
    tdist.batch_isend_irecv = batch_isend_irecv


def _rank(rank: int, world: int, port: int, a) -> None:
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FM_COMM_MODE="single")
    _install_relay()
    from fast_tffm_amd.data.synthetic import CriteoSynth
    from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
    from fast_tffm_amd.ops import kernels as K
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cuda:0")
    cfg = FMConfig(vocabulary_size=a.slots_per_gpu * world, factor_num=64, loss_type="logistic", batch_size=a.batch,
                   init_value_range=0.01, seed=42, opt=K.OptConfig("adagrad", lr=0.01), mode="shard",
                   prefetch_rows="on")
    m = FactorizationMachine(cfg, device="cuda:0", dist=ctx)
    gen = CriteoSynth(cfg.vocabulary_size, seed=1000 + rank, device="cuda:0")
    pool = [gen.batch(a.batch) for _ in range(4)]
    n = a.steps + 3
    t0 = None
    for i in range(n):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        m.train_step(pool[i % 4], pool[(i + 1) % 4], pool[(i + 2) % 4])
    torch.cuda.synchronize()
    loss = m.train_step(pool[n % 4]).mean_loss()
    print(f"[relay_bench] rank {rank}/{world}: {(time.perf_counter() - t0) / a.steps * 1e3:.1f} ms/step "
          f"(host relay, not a measurement) loss={loss:.5f} early_steps={m._exchange.early_steps}", flush=True)
    m.close()
    fmdist.shutdown()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--slots-per-gpu", type=int, default=62_500_000)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(a.world, port, a), nprocs=a.world, join=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
