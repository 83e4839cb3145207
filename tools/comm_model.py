#!/usr/bin/env python3
"""Communication model of the multi-GPU bench configs (bytes per rank per step, predicted time).

For N = 1/2/4/8 ranks it builds the synthetic Criteo-shaped batches every rank would train on
(bench.py: seed 1000 + rank, B examples per rank, 125M hashed slots per rank), measures the
quantities the exchange's traffic depends on -- unique keys per rank U, their split over the
owners (id % N), the rows a rank receives requests for, and the "dirty" share of the early row
exchange (rows a step requests that the previous step updated: they are re-sent after the
update) -- and turns them into bytes per rank per step with the wire layout of
parallel/exchange.py / ops/kernels.py WireFormat:

  row-sharded (bench preset k64, fp32 wire):  ids 4 B + rows rb + gradient rows 4 * g_words, to the
                                              other ranks only (own rows: self rows, no traffic)
                                              + the dirty re-send (rb per dirty row)
  dp_dense (preset k64_dp_dense, V = 1M):     reduce-scatter of the [V, Kp+4] fp32 gradient
                                              buffer + all-gather of the updated [v | w] rows

Predicted time: bytes on the critical path / per-rank link bandwidth, with N - 1 xGMI links in
use by an all-to-all (each peer pair has one direct link) and ring collectives bound by one
link (--link-gbs, unidirectional GB/s per link; MI355X: 7 links per GPU).  The critical path of
the sharded step holds the dirty re-send and the gradient all-to-all (the clean rows travel
early, during the previous step); the model reports both the total and the critical-path bytes.
The first SCALE run of the driver checks these numbers (bench.py prints comm_bytes_per_rank,
counted by the exchange itself).

Usage: python tools/comm_model.py [--batch 131072] [--ranks 1 2 4 8] [--link-gbs 64] [--step-ms 0.67]
"""

from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402


def unique_keys(vocab: int, B: int, seed: int) -> torch.Tensor:
    b = CriteoSynth(vocab, seed=seed).batch(B)
    return torch.unique(b.ids.to(torch.int64))


def shard_model(N: int, B: int, slots: int, Kp: int = 64):
    vocab = slots * N
    rb = Kp * 4 + 16          # fp32 wire row: [v | w, pad]
    gb = (Kp + 4) * 4         # fp32 gradient row
    # two consecutive steps of every rank (pool cycling: batch t on rank r = seed 1000 + r, the
    # bench cycles a pool; consecutive pool entries come from the same generator stream)
    gens = [CriteoSynth(vocab, seed=1000 + r) for r in range(N)]
    step0 = [torch.unique(g.batch(B).ids.to(torch.int64)) for g in gens]
    step1 = [torch.unique(g.batch(B).ids.to(torch.int64)) for g in gens]
    me = 0
    u = step1[me]
    owner = u % N
    U = u.numel()
    to_others = int((owner != me).sum())
    # requests rank `me` receives (as owner) from the other ranks
    recv_others = sum(int((step1[r] % N == me).sum()) for r in range(N) if r != me)
    # dirty: rows of step 1 requested from me by others that step 0 updated (any rank requested them)
    upd0 = torch.unique(torch.cat(step0))
    dirty_send = 0
    for r in range(N):
        if r == me:
            continue
        req = step1[r][step1[r] % N == me]
        dirty_send += int(torch.isin(req, upd0).sum())
    ids_b = 4 * to_others
    rows_b = rb * recv_others
    grads_b = gb * to_others
    patch_b = rb * dirty_send
    total = ids_b + rows_b + grads_b + patch_b
    critical = patch_b + grads_b
    return dict(N=N, U=U, to_others=to_others, recv_others=recv_others, dirty=dirty_send, ids=ids_b, rows=rows_b,
                grads=grads_b, patch=patch_b, total=total, critical=critical)


def dp_touched(N: int, B: int, V: int = 1_000_000, blocks=(16, 256, 4096)):
    """Union over the N ranks' batches of the touched rows of the replicated V-row table, and the share
    of row blocks (of each size) holding at least one touched row: what exchanging only touched rows
    / touched blocks could save."""
    t = torch.zeros(V, dtype=torch.bool)
    for r in range(N):
        t[CriteoSynth(V, seed=1000 + r).batch(B).ids.to(torch.int64)] = True
    out = {"rows": float(t.float().mean())}
    for bs in blocks:
        tt = torch.cat([t, torch.zeros((-V) % bs, dtype=torch.bool)])
        out[bs] = float(tt.view(-1, bs).any(1).float().mean())
    return out


def dp_dense_model(N: int, V: int = 1_000_000, Kp: int = 64):
    buf = V * (Kp + 4) * 4
    rows = V * (Kp + 1) * 4
    rs = (N - 1) * buf // N
    ag = (N - 1) * rows // N
    return dict(N=N, reduce_scatter=rs, all_gather=ag, total=rs + ag, allreduce_equiv=2 * (N - 1) * buf // N)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--slots", type=int, default=125_000_000)
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--link-gbs", type=float, default=64.0, help="unidirectional GB/s per xGMI link (effective)")
    ap.add_argument("--step-ms", type=float, default=0.67, help="measured 1-GPU step (compute) time")
    ap.add_argument("--stale-step-ms", type=float, default=None,
                    help="measured world-1 step of the bounded-staleness executor (bench.py --mode shard "
                         "--staleness 1): its compute, every row through the owner gather / apply")
    ap.add_argument("--dp-fwd-ms", type=float, default=0.20, help="dp_dense forward at world 1")
    ap.add_argument("--dp-bwd-ms", type=float, default=0.45, help="dp_dense backward (EMIT_TABLE) at world 1")
    ap.add_argument("--dp-apply-ms", type=float, default=0.10, help="dp_dense dense_apply of all V rows at world 1")
    ap.add_argument("--dp-blocks", type=int, default=4, help="dp_dense pipeline blocks (FM_DP_BLOCKS)")
    a = ap.parse_args()
    mb = 1e6
    print(f"row-sharded k=64 fp32 wire, B={a.batch}/rank, {a.slots / 1e6:.0f}M slots/rank; "
          f"link {a.link_gbs:.0f} GB/s/direction; compute {a.step_ms:.2f} ms/step")
    print(f"{'N':>2} {'U':>8} {'ids->':>8} {'req<-':>8} {'dirty':>8} {'ids MB':>7} {'rows MB':>8} {'grads MB':>9} "
          f"{'patch MB':>9} {'total MB':>9} {'crit MB':>8} {'t_crit ms':>9} {'pred ms':>8} {'pred eff':>8}")
    for N in a.ranks:
        d = shard_model(N, a.batch, a.slots)
        links = max(N - 1, 1)
        t_crit = d["critical"] / (links * a.link_gbs * 1e9) * 1e3 if N > 1 else 0.0
        t_all = d["total"] / (links * a.link_gbs * 1e9) * 1e3 if N > 1 else 0.0
        # the clean early rows overlap the compute; the critical-path bytes add to it
        pred = max(a.step_ms + t_crit, t_all)
        print(f"{N:>2} {d['U']:>8} {d['to_others']:>8} {d['recv_others']:>8} {d['dirty']:>8} {d['ids'] / mb:>7.1f} "
              f"{d['rows'] / mb:>8.1f} {d['grads'] / mb:>9.1f} {d['patch'] / mb:>9.1f} {d['total'] / mb:>9.1f} "
              f"{d['critical'] / mb:>8.1f} {t_crit:>9.3f} {pred:>8.3f} {a.step_ms / pred:>8.2f}")
    print()
    stale_ms = a.stale_step_ms or a.step_ms
    print(f"bounded staleness (staleness = 1): no dirty patch; step t-1's gradient all-to-all + owner apply and the "
          f"gather + all-to-all of step t+1's rows run beside step t's compute ({stale_ms:.3f} ms/step at world 1, "
          f"every row through the owner gather / apply), so no exchange byte is on the critical path while that "
          f"chain fits a step:  pred = max(compute, bytes / links)")
    print(f"{'N':>2} {'total MB':>9} {'t_all ms':>9} {'pred ms':>8} {'eff vs sync N=1':>15} {'eff vs stale N=1':>16}")
    for N in a.ranks:
        d = shard_model(N, a.batch, a.slots)
        links = max(N - 1, 1)
        tot = d["ids"] + d["rows"] + d["grads"]  # (no patch)
        t_all = tot / (links * a.link_gbs * 1e9) * 1e3 if N > 1 else 0.0
        pred = max(stale_ms, t_all)
        print(f"{N:>2} {tot / mb:>9.1f} {t_all:>9.3f} {pred:>8.3f} {a.step_ms / pred:>15.2f} {stale_ms / pred:>16.2f}")
    print()
    print("dp_dense k=64 (V = 1M replicated, fp32 gradient buffer): reduce-scatter + sharded apply + all-gather")
    print(f"  compute at world 1: forward {a.dp_fwd_ms:.3f} ms, backward {a.dp_bwd_ms:.3f} ms, "
          f"apply {a.dp_apply_ms:.3f} ms; P = {a.dp_blocks} row blocks")
    print("  serial:    fwd + bwd + RS + apply + AG")
    print("  pipelined: fwd + max(bwd, bwd/P + RS) + apply/P + AG   (RS(p) beside backward piece p+1, apply(p) beside")
    print("             RS(p+1), AG(p) beside apply(p+1); the forward reads every block's updated rows, so the")
    print("             all-gather cannot run beside the next step in a synchronous step)")
    print(f"{'N':>2} {'RS MB':>8} {'AG MB':>8} {'total MB':>9} {'allreduce MB':>12} {'t ring ms':>9} {'serial ms':>9} "
          f"{'pipe ms':>8} {'max+10% ms':>10}")
    for N in a.ranks:
        d = dp_dense_model(N)
        # RCCL runs its rings over every peer link of the fully connected mesh (N - 1 links)
        bw = max(N - 1, 1) * a.link_gbs * 1e9
        t = d["total"] / bw * 1e3
        rs, ag = d["reduce_scatter"] / bw * 1e3, d["all_gather"] / bw * 1e3
        comp = a.dp_fwd_ms + a.dp_bwd_ms + a.dp_apply_ms / max(N, 1)
        serial = comp + rs + ag
        P = a.dp_blocks if N > 1 else 1
        pipe = (a.dp_fwd_ms + max(a.dp_bwd_ms, a.dp_bwd_ms / P + rs) + a.dp_apply_ms / max(N, 1) / P + ag)
        print(f"{N:>2} {d['reduce_scatter'] / mb:>8.1f} {d['all_gather'] / mb:>8.1f} {d['total'] / mb:>9.1f} "
              f"{d['allreduce_equiv'] / mb:>12.1f} {t:>9.3f} {serial:>9.3f} {pipe:>8.3f} {1.1 * max(comp, t):>10.3f}")
    print()
    print("dp_dense: touched rows (union over the ranks' batches) and touched row blocks -- the bytes an exchange of")
    print("only touched blocks / rows would move (RS + AG scale with the exchanged share; row-granular exchange")
    print("needs the per-rank counts on the host before the collectives: one host sync per step)")
    print(f"{'N':>2} {'rows':>6} {'blk16':>6} {'blk256':>7} {'blk4096':>8} {'blocks MB':>10} {'rows MB':>8} "
          f"{'rows pipe ms':>12} {'bf16-RS rows pipe ms':>20}")
    for N in a.ranks:
        d = dp_dense_model(N)
        tch = dp_touched(N, a.batch)
        bw = max(N - 1, 1) * a.link_gbs * 1e9
        blk_b = d["total"] * tch[4096]
        # row-granular: the touched rows' data + one int32 id per exchanged row
        row_b = d["total"] * tch["rows"] + 2 * 4 * (N - 1) * 1_000_000 * tch["rows"] / max(N, 1)
        P = a.dp_blocks if N > 1 else 1
        def pipe(rs_b, ag_b):
            rs, ag = rs_b / bw * 1e3, ag_b / bw * 1e3
            return a.dp_fwd_ms + max(a.dp_bwd_ms, a.dp_bwd_ms / P + rs) + a.dp_apply_ms / max(N, 1) / P + ag
        rs_rows = d["reduce_scatter"] * tch["rows"]
        ag_rows = d["all_gather"] * tch["rows"]
        print(f"{N:>2} {tch['rows']:>6.3f} {tch[16]:>6.3f} {tch[256]:>7.3f} {tch[4096]:>8.3f} {blk_b / mb:>10.1f} "
              f"{row_b / mb:>8.1f} {pipe(rs_rows, ag_rows):>12.3f} {pipe(rs_rows / 2, ag_rows):>20.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
