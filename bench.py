#!/usr/bin/env python3
"""Headline benchmark: Criteo-shaped FM training throughput on MI355X.

Metric (BASELINE.json): examples/sec for the whole node, Criteo-shaped FM k=64,
at 1/2/4/8 MI355X.  One process per GPU (torchrun), RCCL over xGMI.

Workload per step and rank (weak scaling: per-GPU work is fixed as N grows):
  * B examples x 39 features (13 bucketized integer + 26 categorical Criteo
    fields, Zipf value popularity), synthetic, generated on the device before
    timing (a pool of distinct batches is cycled);
  * FM k=64 (default preset k64): fp32 factor table, fp32 arithmetic and fp32
    Adagrad slots -- the reference's precision (tffm/fm_model.py:269-284);
    hashed vocabulary of 125M slots per GPU (1B slots at N=8), row-sharded over
    the GPUs with RCCL all-to-all for lookups and gradients (mode "shard", fp32
    rows on the wire); N=1 runs the local single-GPU path.  `--preset k64_bf16`
    is the same model with a bf16 table (secondary number, profiles/);
  * the timed step is the full training step: id -> key, dedup, (a2a), fused
    forward + loss, fused backward + Adagrad update, (a2a + owner update).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] ...
        (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402
from fast_tffm_amd.parallel import dist as fmdist  # noqa: E402


def native_hashes() -> dict:
    from fast_tffm_amd.ops import native

    return native.build_hashes()

PRESETS = {
    # BASELINE.json headline: FM k=64 Criteo-shaped, row-sharded 1B slots at N=8
    "k64": dict(k=64, dtype="fp32", opt="adagrad", mode="auto", slots_per_gpu=125_000_000),
    # the headline model with a bf16 factor table (fp32 compute, accumulation and optimizer state)
    "k64_bf16": dict(k=64, dtype="bf16", opt="adagrad", mode="auto", slots_per_gpu=125_000_000),
    # BASELINE config 2: k=16 bf16 table
    "k16_bf16": dict(k=16, dtype="bf16", opt="adagrad", mode="auto", slots_per_gpu=125_000_000),
    # BASELINE config 3: k=64 data-parallel, dense all-reduce (small replicated vocabulary)
    "k64_dp_dense": dict(k=64, dtype="fp32", opt="adagrad", mode="dp_dense", slots_per_gpu=None,
                         vocab=1_000_000),
    # BASELINE config 5: k=128 fp8 factor table (OCP e4m3 + per-row scale) + fused FTRL
    "k128_fp8_ftrl": dict(k=128, dtype="fp8", opt="ftrl", mode="auto", slots_per_gpu=62_500_000),
    # same with a bf16 table (reference point for the fp8 one)
    "k128_ftrl": dict(k=128, dtype="bf16", opt="ftrl", mode="auto", slots_per_gpu=62_500_000),
    # BASELINE config 1: 2nd-order FM k=4 on a tiny a1a-shaped libsvm set, CPU, world_size 1
    # (plumbing: text -> C++ parser -> OpenMP CPU kernels); data goes through the real reader
    "a1a_cpu": dict(k=4, dtype="fp32", opt="adagrad", mode="local", slots_per_gpu=None, vocab=124,
                    device="cpu", data="a1a", batch=1605),
}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="examples per GPU per step (default 131072)")
    ap.add_argument("--preset", default="k64", choices=sorted(PRESETS))
    ap.add_argument("--slots-per-gpu", type=int, default=None, help="override hashed slots per GPU")
    ap.add_argument("--pool", type=int, default=16, help="distinct synthetic batches cycled")
    ap.add_argument("--alpha", type=float, default=1.1, help="Zipf exponent of field values")
    ap.add_argument("--mode", default=None, help="override step mode (local|shard|dp|dp_dense)")
    ap.add_argument("--microbatches", type=int, default=0,
                    help="row-sharded step: parts per batch overlapping the exchange (0/1 = one part)")
    ap.add_argument("--prefetch-rows", default="auto", choices=["auto", "on", "off"],
                    help="row-sharded step: exchange next step's rows early, patch the updated ones (auto: N > 1)")
    ap.add_argument("--overlap-grads", default="auto", choices=["auto", "on", "off"],
                    help="row-sharded step: split backward, first half's gradient rows sent early (auto: off)")
    ap.add_argument("--comm-dtype", default="auto", choices=["auto", "fp32", "bf16"],
                    help="row-sharded wire rows (auto = table storage dtype; bf16 rounds fp32 rows for transport)")
    ap.add_argument("--staleness", type=int, default=0, choices=[0, 1],
                    help="row-sharded step: 0 = synchronous (default), 1 = bounded staleness (the reference's "
                         "asynchronous updates, deterministic: rows read one step stale, exchange + apply overlap)")
    ap.add_argument("--stochastic-rounding", default="on", choices=["on", "off"],
                    help="bf16 / fp8 tables: stochastically rounded row stores (the training default)")
    ap.add_argument("--profile-steps", type=int, default=0, help="also emit a torch.profiler trace")
    ap.add_argument("--graph", type=int, default=0,
                    help="local step: 0 = eager lookahead pipeline (next batch's dedup overlaps this step; "
                         "measured fastest), 1 = the same pipeline as a hipGraph ring")
    a = ap.parse_args()

    p = dict(PRESETS[a.preset])
    a.batch = a.batch or p.get("batch", 131072)
    mode = a.mode or p["mode"]
    if mode not in ("auto", "local") or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # 8 HIP hardware queues for the multi-rank step (parallel/dist.py ensure_hw_queues; the
        # single-GPU step keeps HIP's default 4).  Must be set before HIP initialises.
        fmdist.ensure_hw_queues()
    # bounded collective timeout: a hang in the multi-GPU bench exits non-zero after
    # FM_PG_TIMEOUT seconds (RCCL watchdog) instead of holding the node for 30 minutes
    ctx = fmdist.init_distributed(force_pg=mode not in ("auto", "local"), device=p.get("device"),
                                  timeout_s=float(os.environ.get("FM_PG_TIMEOUT", "300")))
    W, rank = ctx.world, ctx.rank
    if W != a.gpus:  # (the __main__ guard already refused this; library callers of main() too)
        print(f"[bench] error: --gpus {a.gpus} but WORLD_SIZE={W}", file=sys.stderr)
        return 2
    dev = ctx.device
    if dev.type != "cuda":
        print("[bench] no GPU visible: running on CPU (not a valid measurement)", file=sys.stderr)
    slots = a.slots_per_gpu or p.get("slots_per_gpu")
    vocab = slots * W if slots else p["vocab"]
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn}[p["dtype"]]
    opt = K.OptConfig(p["opt"], lr=0.01 if p["opt"] == "adagrad" else 0.05, l1=0.001, l2=0.001, beta=1.0,
                      initial_accumulator=0.1)
    cfg = FMConfig(vocabulary_size=vocab, factor_num=p["k"], loss_type="logistic", batch_size=a.batch,
                   init_value_range=0.01, seed=42, dtype=dtype, opt=opt, mode=mode, comm_dtype=a.comm_dtype,
                   microbatches=a.microbatches, prefetch_rows=a.prefetch_rows,
                   overlap_grads=a.overlap_grads, stochastic_rounding=a.stochastic_rounding == "on",
                   staleness=a.staleness)
    t0 = time.time()
    model = FactorizationMachine(cfg, device=dev, dist=ctx if W > 1 or mode not in ("auto", "local") else None)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] {model.table.memory_report()} (init {time.time() - t0:.1f}s), mode={model.mode}, "
              f"vocab={vocab}, B/gpu={a.batch}", file=sys.stderr)

    if p.get("data") == "a1a":  # libsvm text through the C++ parser (tools/make_sample_data.py shape)
        import tempfile

        from fast_tffm_amd.data.reader import load_file_batch
        from fast_tffm_amd.data.synthetic import write_libsvm

        pool = []
        with tempfile.TemporaryDirectory() as td:
            for i in range(max(1, a.pool)):
                path = os.path.join(td, f"a1a_{i}")
                write_libsvm(path, a.batch, shape="a1a", seed=1000 * rank + i, weights_path=None)
                pool.append(load_file_batch([path], None, vocab, False, 4).to(dev))
    else:
        gen = CriteoSynth(vocab, alpha=a.alpha, seed=1000 + rank, device=dev)
        pool = [gen.batch(a.batch) for _ in range(max(1, a.pool))]
    if dev.type == "cuda":
        torch.cuda.synchronize()
    graphed = False
    if a.graph and dev.type == "cuda" and model.mode == "local":
        # lookahead hipGraph ring: step k replays one graph running this batch's fwd/bwd and,
        # concurrently, the dedup of batch k+1.  The synthetic "loader" writes each pool batch
        # into a ring buffer once (a staging pipeline would H2D-copy into them)
        n = len(pool) + (len(pool) % 2)
        bufs = model.lookahead_graph_buffers(pool[0], n)
        for i, dst in enumerate(bufs):
            src = pool[i % len(pool)]
            for d, s in ((dst.labels, src.labels), (dst.offsets, src.offsets), (dst.ids, src.ids)):
                d.copy_(s)
        pool = bufs
        torch.cuda.synchronize()
        graphed = True
    if rank == 0:
        from fast_tffm_amd.ops import kernels as Kd

        dd = Kd.dedup(pool[0].ids if pool[0].ids.dtype == torch.int32 else pool[0].ids.int(), key_bits=32)
        print(f"[bench] batch stats: nnz={pool[0].nnz} unique={dd.sync()} graph={graphed}", file=sys.stderr)

    # the step after step i uses pool[(i + 1) % len(pool)]: pass it as lookahead (the sharded
    # executor dedups / exchanges ids of the next batch while this step computes)
    def nxt(i):
        return pool[(i + 1) % len(pool)]

    def nxt2(i):  # two batches of lookahead (the sharded executor's depth-2 pipeline)
        return pool[(i + 2) % len(pool)] if len(pool) > 2 else None

    for i in range(a.warmup):
        model.train_step(pool[i % len(pool)], nxt(i), nxt2(i))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()

    ex = model._exchange
    comm0 = getattr(ex, "bytes_sent", 0)
    t_start = time.perf_counter()
    last = None
    for i in range(a.steps):
        last = model.train_step(pool[(a.warmup + i) % len(pool)], nxt(a.warmup + i), nxt2(a.warmup + i))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed_own = time.perf_counter() - t_start
    K.check_device_errors(dev)  # (kernels' sticky error word, e.g. a failed sort look-back: exit non-zero)
    elapsed = ctx.all_reduce_scalar(elapsed_own, op="max")
    elapsed_min = ctx.all_reduce_scalar(elapsed_own, op="min")
    # bytes this rank put on the wire to OTHER ranks per timed step (all-to-all rows / ids /
    # gradients, all-reduce / all-gather payloads: parallel/exchange.py accounting), max over ranks
    comm_own = (getattr(ex, "bytes_sent", 0) - comm0) / max(a.steps, 1)
    comm_max = ctx.all_reduce_scalar(comm_own, op="max")
    import torch.distributed as tdist

    rccl_world = tdist.get_world_size(ctx.group) if (ctx.group is not None and tdist.is_initialized()) else 1
    comm_backend = tdist.get_backend(ctx.group) if (ctx.group is not None and tdist.is_initialized()) else None

    loss = last.mean_loss() if last is not None else float("nan")
    if a.profile_steps and rank == 0:
        from fast_tffm_amd.utils.trace import profile_steps

        profile_steps(lambda i: model.train_step(pool[i % len(pool)]), a.profile_steps,
                      os.path.join(ROOT, "gpurun_out", "bench_trace.json"))

    ex_total = a.batch * W * a.steps
    value = ex_total / elapsed
    ms = elapsed / a.steps * 1e3
    if rank == 0:
        par = ("rowshard%d" % W) if model.mode == "shard" else (model.mode + str(W) if W > 1 else "single")
        print(f"[bench] loss={loss:.5f} ms/step={ms:.3f} ex/s={value:.4g}", file=sys.stderr)
        line = json.dumps({
            "metric": ("examples/sec (whole node), Criteo-shaped FM k=%d" % p["k"]) if p.get("data") != "a1a"
            else "examples/sec, a1a-shaped FM k=%d on CPU (plumbing config)" % p["k"],
            "value": value,
            "unit": "examples/s",
            "n_gpus": W,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # the table's storage dtype (bf16 / fp8 tables: fp32 arithmetic, accumulators and
            # optimizer state; fp32: everything fp32)
            "dtype": p["dtype"],
            "data": ("synthetic Criteo-shaped (39 fields, Zipf a=%.2f), random-init weights" % a.alpha)
            if p.get("data") != "a1a" else "synthetic a1a-shaped libsvm text (123 features), parsed",
            "config": {
                "model": "FM k=%d, %s table + %s, hashed vocab %d (%d/GPU)" % (
                    p["k"], p["dtype"], p["opt"], vocab, vocab // W if model.mode == "shard" else vocab),
                "global_batch": a.batch * W,
                "seq_len": 39,
                "parallelism": par,
                "wire": str(model._exchange.wire.dtype).replace("torch.", "")
                if model.mode == "shard" else None,
                "microbatches": model._exchange.nparts if model.mode == "shard" else None,
                "early_rows": bool(model._exchange.prefetch) if model.mode == "shard" else None,
                "split_grads": bool(model._exchange.overlap_grads) if model.mode == "shard" else None,
                "comm": getattr(model._exchange, "comm_mode", None),
                "staleness": getattr(model._exchange, "staleness", 0) if model.mode == "shard" else None,
                "seg_lookup": K.seg_lookup_enabled() if model.mode == "shard" else None,
                "lookahead": (2 if os.environ.get("FM_LOCAL_DEPTH2", "1") != "0" and len(pool) > 2 else 1)
                if model.mode == "local" and dev.type == "cuda" and not graphed else None,
                "pool": len(pool),
                # world size of the process group the step's collectives ran on (RCCL on GPUs)
                "rccl_world": rccl_world,
                "comm_backend": comm_backend,
                # timed-loop wall time per step, slowest / fastest rank (value uses the slowest)
                "per_rank_ms": {"max": elapsed / a.steps * 1e3, "min": elapsed_min / a.steps * 1e3},
                "comm_bytes_per_rank": int(round(comm_max)),
                "native_build": native_hashes(),
            },
        })
        sys.stdout.flush()
        os.write(_RESULT_FD, (line + "\n").encode())
    fmdist.shutdown()
    return 0


# stdout carries exactly one line, the JSON result of rank 0: everything else the process
# writes to fd 1 -- including the C++ libraries' own messages (gloo prints its connection
# lines there when the CPU side-group is created) -- goes to stderr
_RESULT_FD = 1


def _launch_guard(argv: list[str]) -> int | None:
    """Multi-GPU invocations without a launcher.  ``--gpus N`` (N > 1) with no torchrun
    environment: start the N ranks here through ``torch.distributed.run`` (one process per GPU,
    rendezvous on 127.0.0.1, like the driver's own launch) and return its exit code -- this
    process never touches the GPU (``import torch`` does not initialise HIP), so the ranks own
    the devices.  ``--gpus N`` disagreeing with an existing WORLD_SIZE is an error (exit 2): a
    1-rank measurement must never be reported as an N-GPU one.  None: run in this process."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    known, _ = pre.parse_known_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != known.gpus:
            print(f"[bench] error: --gpus {known.gpus} but WORLD_SIZE={env_world} (launch {known.gpus} ranks, or "
                  f"pass --gpus {env_world})", file=sys.stderr)
            return 2
        return None
    if known.gpus <= 1:
        return None
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(known.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {known.gpus} ranks: {' '.join(cmd)}", file=sys.stderr)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


if __name__ == "__main__":
    _rc = _launch_guard(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)
    sys.exit(main())
