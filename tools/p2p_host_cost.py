"""Host cost of issuing one split-backward piece: 2 (W - 1) Python P2P ops vs one list all-to-all.

RCCL world 1 on one GPU (the only world a 1-GPU box has), so both forms are posed against the own rank:
  p2p   2 (W - 1) ``P2POp``s (W - 1 sends + W - 1 receives, all to rank 0) in one ``batch_isend_irecv``
  a2a   one ``all_to_all`` over the W per-peer views (a world-1 group takes a list of one; the W views are
        still sliced, as the executor slices them)
Prints the host microseconds per piece (issue only: the device work is waited for outside the timing).

    python tools/p2p_host_cost.py --peers 8 --iters 200
"""

import argparse
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rows", type=int, default=4096)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    W, R = a.peers, a.rows
    send = torch.randn(W * R, 64, device="cuda:0")
    recv = torch.empty_like(send)

    def p2p():
        ops = []
        for q in range(1, W):
            ops.append(dist.P2POp(dist.isend, send[q * R:(q + 1) * R], 0))
            ops.append(dist.P2POp(dist.irecv, recv[q * R:(q + 1) * R], 0))
        return dist.batch_isend_irecv(ops)

    def a2a():
        ins = [send[q * R:(q + 1) * R] for q in range(W)]
        outs = [recv[q * R:(q + 1) * R] for q in range(W)]
        return [dist.all_to_all(outs[:1], ins[:1], async_op=True)]

    for name, fn in (("p2p", p2p), ("a2a", a2a), ("p2p", p2p), ("a2a", a2a)):
        for _ in range(10):
            for w in fn():
                w.wait()
        torch.cuda.synchronize()
        t = 0.0
        for _ in range(a.iters):
            t0 = time.perf_counter()
            ws = fn()
            t += time.perf_counter() - t0
            for w in ws:
                w.wait()
            torch.cuda.synchronize()
        print(f"{name}  W={W}  host us per piece {1e6 * t / a.iters:8.1f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
