"""bench.py output contract (one JSON line with the driver's keys), exercised on CPU with a
tiny configuration; the real measurement runs on the GPU (see profiles/)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(args):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("args", [["--steps", "2", "--warmup", "1", "--batch", "256", "--slots-per-gpu", "20000"],
                                  ["--preset", "a1a_cpu", "--steps", "2", "--warmup", "1"]])
def test_bench_prints_one_json_line(args):
    d = _run(args)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "weak"
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])


def test_bench_two_ranks_one_json_line():
    """The driver's N>1 launch (torch.distributed.run, one process per device, 127.0.0.1):
    stdout holds exactly rank 0's JSON line (the gloo side-group's connection messages and
    every other rank's output go to stderr), n_gpus / global_batch / parallelism follow the
    world size.  CPU + gloo here; the same path runs RCCL on MI355X."""
    import socket

    from ports import free_port

    port = free_port()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "256", "--slots-per-gpu", "20000",
                        "--preset", "k64"],  # (bf16 storage wires of the default preset are a GPU path)
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert KEYS <= set(d) and d["n_gpus"] == 2 and d["config"]["global_batch"] == 512
    assert d["config"]["parallelism"] == "rowshard2" and d["config"]["early_rows"] and d["config"]["split_grads"]
    assert d["config"]["rccl_world"] == 2 and d["config"]["comm_backend"] == "gloo"
    assert d["config"]["per_rank_ms"]["max"] >= d["config"]["per_rank_ms"]["min"] > 0
    assert d["config"]["comm_bytes_per_rank"] > 0


def test_bench_self_launches_ranks():
    """``bench.py --gpus 2`` with no launcher environment starts the 2 ranks itself (through
    torch.distributed.run, before any device call) instead of measuring one process."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--batch", "256", "--slots-per-gpu", "20000"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["rccl_world"] == 2 and d["config"]["global_batch"] == 512


def test_bench_world_mismatch_exits_nonzero():
    """An existing WORLD_SIZE that disagrees with --gpus is refused (exit 2, no JSON line)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "0", "--batch", "64", "--slots-per-gpu", "2000"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert not r.stdout.strip()
    assert "WORLD_SIZE" in r.stderr
