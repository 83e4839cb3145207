"""Checkpoint / resume, and conversion to the reference's table layout.

Reference: ``tf.train.Saver`` bundles in ``log_dir`` written by
``CheckpointSaverHook(save_steps)`` (run_tffm.py:213-216); variables
``vocab_block_{i}`` ``[V // N + 1, K + 1]`` (column 0 = w), their Adagrad slots
and ``global_step``; ``MonitoredTrainingSession`` restores the latest
checkpoint automatically; ``generate`` uses ``get_checkpoint_state(log_dir)``.

Layout here (one directory per step, one file per table shard)::

    log_dir/checkpoint                         TF-style index: model_checkpoint_path: "model.ckpt-<step>"
    log_dir/model.ckpt-<step>/meta.json        step, shapes, optimizer, world, reader position
    log_dir/model.ckpt-<step>/shard-RRRRR-of-WWWWW.safetensors
        w [rows] fp32, v [rows, K] (table dtype), s0w/s0v (Adagrad acc / FTRL n),
        s1w/s1v (FTRL z); local row r of shard s holds global id r * W + s.

Every rank writes only its own shard (replicated modes: rank 0 writes the
single table); rank 0 writes meta.json and the index after a barrier, so the
index never points at a partial checkpoint.  Restore re-shards on the fly when
the world size changed.  ``export_reference_blocks``/``import_reference_blocks``
convert to/from ``vocab_block_{i}`` arrays in the reference's mod layout.
"""

from __future__ import annotations

import glob
import json
import os
import re
import shutil

import numpy as np
import torch
from safetensors import safe_open
from safetensors.torch import load_file, save_file  # noqa: F401  (small files / tools)

FORMAT = "fast_tffm_amd/ckpt-v1"
INDEX = "checkpoint"


def _shard_name(rank: int, world: int) -> str:
    return f"shard-{rank:05d}-of-{world:05d}.safetensors"


def latest_checkpoint(log_dir: str | None) -> str | None:
    """Path of the newest complete checkpoint directory in ``log_dir`` (or None)."""
    if not log_dir or not os.path.isdir(log_dir):
        return None
    idx = os.path.join(log_dir, INDEX)
    if os.path.exists(idx):
        with open(idx) as f:
            for line in f:
                m = re.match(r'model_checkpoint_path:\s*"(.*)"', line.strip())
                if m:
                    p = m.group(1)
                    p = p if os.path.isabs(p) else os.path.join(log_dir, p)
                    if os.path.exists(os.path.join(p, "meta.json")):
                        return p
    cands = sorted(glob.glob(os.path.join(log_dir, "model.ckpt-*", "meta.json")),
                   key=lambda p: int(re.search(r"model\.ckpt-(\d+)", p).group(1)))
    return os.path.dirname(cands[-1]) if cands else None


# safetensors dtype names
_ST_DTYPE = {torch.float32: "F32", torch.bfloat16: "BF16", torch.uint8: "U8", torch.int64: "I64",
             torch.int32: "I32", torch.float16: "F16"}
CHUNK_BYTES = 256 << 20   # rows move device -> file (and back) in chunks of about this size


def _table_sources(table) -> dict:
    """name -> (dtype, shape, chunk(r0, r1) -> tensor of rows [r0, r1)) of a table shard.

    Chunked so that a checkpoint of a 125M-row shard never holds more than one chunk of
    any table tensor in host memory (nor a full-size dequantised copy on the device)."""
    K, n = table.K, table.saved_rows

    def rows(t, cols=None):
        return lambda r0, r1: (t[r0:r1] if cols is None else t[r0:r1, :cols])

    src = {"w": (torch.float32, (n,), rows(table.w)),
           "v": (table.dtype if not table.fp8 else torch.float32, (n, K),
                 (lambda r0, r1: table.dense_v(slice(r0, r1))[:, :K])
                 if table.fp8 else rows(table.v, K)),
           "s0w": (torch.float32, (n,), rows(table.s0w)),
           "s0v": (torch.float32, (n, K), rows(table.s0v, K))}
    if table.fp8:  # exact fp8 payload + scales next to the portable fp32 values
        src["v_fp8"] = (torch.uint8, (n, table.Kp), rows(table.v.view(torch.uint8)))
        src["v_scale"] = (torch.float32, (n,), rows(table.scale))
    if table.s1v is not None:
        src["s1w"] = (torch.float32, (n,), rows(table.s1w))
        src["s1v"] = (torch.float32, (n, K), rows(table.s1v, K))
    return src


def write_safetensors_streamed(path: str, sources: dict, metadata: dict | None = None) -> None:
    """Write a safetensors file from row-chunk producers (see ``_table_sources``): the header
    first (8-byte length + JSON, data aligned to 8 bytes), then each tensor chunk by chunk."""
    header, off, plan = {}, 0, []
    for name, (dtype, shape, chunk) in sources.items():
        esz = torch.tensor([], dtype=dtype).element_size()
        nbytes = int(np.prod(shape)) * esz if len(shape) else esz
        header[name] = {"dtype": _ST_DTYPE[dtype], "shape": list(shape), "data_offsets": [off, off + nbytes]}
        plan.append((name, dtype, shape, chunk, nbytes))
        off += nbytes
    if metadata:
        header["__metadata__"] = {k: str(v) for k, v in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - (len(hb) + 8) % 8) % 8)
    with open(path, "wb") as f:
        f.write(len(hb).to_bytes(8, "little"))
        f.write(hb)
        for name, dtype, shape, chunk, nbytes in plan:
            n = shape[0] if shape else 1
            row_bytes = max(1, nbytes // max(n, 1))
            step = max(1, CHUNK_BYTES // row_bytes)
            for r0 in range(0, n, step):
                c = chunk(r0, min(n, r0 + step)).detach()
                c = c.to(dtype).contiguous().cpu() if c.dtype != dtype else c.contiguous().cpu()
                f.write(c.view(torch.uint8).numpy().tobytes())


def _table_tensors(table) -> dict[str, torch.Tensor]:
    """Whole shard tensors on the host (small tables / tests; checkpoints stream instead)."""
    return {k: c(0, shape[0]).detach().to(dt).cpu().contiguous() for k, (dt, shape, c) in _table_sources(table).items()}


def save_checkpoint(model, log_dir: str, step: int, *, reader_state: dict | None = None, ctx=None,
                    max_to_keep: int = 5) -> str:
    """Write a checkpoint of ``model`` (a FactorizationMachine) at ``step``; returns its directory."""
    table = model.table
    rank = ctx.rank if ctx is not None else 0
    world = ctx.world if ctx is not None else 1
    sharded = model.mode == "shard"
    path = os.path.join(log_dir, f"model.ckpt-{step}")
    os.makedirs(path, exist_ok=True)
    ex = getattr(model, "_exchange", None)
    if ex is not None and hasattr(ex, "sync_state"):  # (collective: every rank) sharded optimizer state
        ex.sync_state()
    if sharded or rank == 0:
        shard_rank, shard_world = (table.rank, table.world)
        tmp = os.path.join(path, _shard_name(shard_rank, shard_world) + ".tmp")
        sources = _table_sources(table)
        if getattr(model, "gbias", None) is not None:  # replicated global bias + optimizer state
            for k in ("gbias", "gbias_s0", "gbias_s1"):
                t = getattr(model, k)
                sources[k] = (torch.float32, tuple(t.shape), (lambda t_: lambda r0, r1: t_[r0:r1])(t))
        write_safetensors_streamed(tmp, sources, {"format": FORMAT, "rank": shard_rank, "world": shard_world})
        os.replace(tmp, os.path.join(path, _shard_name(shard_rank, shard_world)))
    # every rank reads its own file subset (reader.py / loader.cpp shard the files by rank),
    # so each rank's reader position is saved and restored separately
    reader_states = {"0": reader_state or {}}
    if ctx is not None and world > 1:
        import torch.distributed as dist

        allrs = [None] * world
        dist.all_gather_object(allrs, reader_state or {}, group=ctx.cpu_group or ctx.group)
        reader_states = {str(r): s for r, s in enumerate(allrs)}
        ctx.barrier()
    if rank == 0:
        meta = {
            "format": FORMAT,
            "global_step": int(step),
            "vocabulary_size": table.vocab_size,
            "factor_num": table.K,
            "dtype": str(table.dtype).replace("torch.", ""),
            "optimizer": table.opt.name,
            "shard_world": table.world,
            "mode": model.mode,
            "loss_type": model.cfg.loss_type,
            "reader_state": reader_state or {},          # rank 0's (single-process readers)
            "reader_states": reader_states,              # per rank
            "reader_world": world,
            "global_bias": float(model.gbias.item()) if getattr(model, "gbias", None) is not None else None,
        }
        with open(os.path.join(path, "meta.json.tmp"), "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(os.path.join(path, "meta.json.tmp"), os.path.join(path, "meta.json"))
        _write_index(log_dir, os.path.basename(path), max_to_keep)
    if ctx is not None and world > 1:
        ctx.barrier()
    return path


def _write_index(log_dir: str, newest: str, max_to_keep: int) -> None:
    ckpts = sorted(glob.glob(os.path.join(log_dir, "model.ckpt-*")),
                   key=lambda p: int(re.search(r"model\.ckpt-(\d+)$", p).group(1)) if re.search(
                       r"model\.ckpt-(\d+)$", p) else -1)
    ckpts = [c for c in ckpts if os.path.exists(os.path.join(c, "meta.json"))]
    if max_to_keep and len(ckpts) > max_to_keep:
        for old in ckpts[:-max_to_keep]:
            shutil.rmtree(old, ignore_errors=True)
        ckpts = ckpts[-max_to_keep:]
    lines = [f'model_checkpoint_path: "{newest}"']
    lines += [f'all_model_checkpoint_paths: "{os.path.basename(c)}"' for c in ckpts]
    tmp = os.path.join(log_dir, INDEX + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(log_dir, INDEX))


def read_meta(ckpt_dir: str) -> dict:
    with open(os.path.join(ckpt_dir, "meta.json")) as f:
        return json.load(f)


def _iter_shards(ckpt_dir: str):
    for p in sorted(glob.glob(os.path.join(ckpt_dir, "shard-*-of-*.safetensors"))):
        m = re.search(r"shard-(\d+)-of-(\d+)\.safetensors$", p)
        yield int(m.group(1)), int(m.group(2)), p


def restore_checkpoint(model, ckpt_dir: str) -> dict:
    """Load ``ckpt_dir`` into ``model``'s (local) table, re-sharding if needed. Returns meta."""
    meta = read_meta(ckpt_dir)
    table = model.table
    if meta["factor_num"] != table.K or meta["vocabulary_size"] != table.vocab_size:
        raise ValueError(f"checkpoint shape (V={meta['vocabulary_size']}, K={meta['factor_num']}) does not match "
                         f"the model (V={table.vocab_size}, K={table.K})")
    K = table.K
    dev = table.device
    direct = os.path.join(ckpt_dir, _shard_name(table.rank, table.world))
    if getattr(model, "gbias", None) is not None:
        first = next(iter(_iter_shards(ckpt_dir)), None)
        if first is not None:
            with safe_open(first[2], framework="pt") as f:
                for k in ("gbias", "gbias_s0", "gbias_s1"):
                    if k in f.keys():
                        getattr(model, k).copy_(f.get_tensor(k).to(getattr(model, k).device))
    if os.path.exists(direct):
        for r0, t in _iter_row_chunks(direct):
            n = t["w"].shape[0]
            _copy_rows(table, slice(r0, r0 + n), t, K, dev)
    else:
        for s_rank, s_world, path in _iter_shards(ckpt_dir):
            for r0, t in _iter_row_chunks(path):
                n = t["w"].shape[0]
                gid = torch.arange(r0, r0 + n, dtype=torch.int64) * s_world + s_rank
                mine = (gid % table.world == table.rank) & (gid < table.vocab_size)
                if not bool(mine.any()):
                    continue
                sel = torch.nonzero(mine).flatten()
                local = torch.div(gid[sel], table.world, rounding_mode="floor")
                _copy_rows(table, local.to(dev), {k: v[sel] for k, v in t.items()}, K, dev)
    model.global_step = int(meta["global_step"])
    if hasattr(model, "sr_reset"):
        model.sr_reset()
    return meta


_ROW_KEYS = ("w", "v", "s0w", "s0v", "s1w", "s1v", "v_fp8", "v_scale")


def _iter_row_chunks(path: str):
    """(first row, {name: rows}) chunks of a shard file's per-row tensors, read lazily."""
    with safe_open(path, framework="pt") as f:
        keys = [k for k in f.keys() if k in _ROW_KEYS]
        n = f.get_slice("w").get_shape()[0]
        row_bytes = sum(4 * int(np.prod(f.get_slice(k).get_shape()[1:] or [1])) for k in keys)
        step = max(1, CHUNK_BYTES // max(row_bytes, 1))
        for r0 in range(0, n, step):
            r1 = min(n, r0 + step)
            yield r0, {k: f.get_slice(k)[r0:r1] for k in keys}


def _copy_rows(table, local_rows, t: dict, K: int, dev) -> None:
    def put(dst, src, cols=False):
        if dst is None or src is None:
            return
        src = src.to(dev, dst.dtype)
        if local_rows is None:
            n = src.shape[0]
            if cols:
                dst[:n, :K] = src
            else:
                dst[:n] = src
        else:
            if cols:
                dst[local_rows, :K] = src
            else:
                dst[local_rows] = src

    put(table.w, t.get("w"))
    if table.fp8 and "v_fp8" in t:
        put(table.v.view(torch.uint8), t["v_fp8"])
        put(table.scale, t["v_scale"])
        # (power-of-two scales + row norms, of the rows this chunk wrote)
        table.adopt_fp8_rows(torch.arange(t["v_scale"].shape[0], device=dev) if local_rows is None else local_rows)
    elif table.fp8:
        if isinstance(local_rows, slice):
            local_rows = torch.arange(local_rows.start, local_rows.stop, device=dev)
        table.set_v(local_rows, t["v"].float())
    else:
        put(table.v, t.get("v"), cols=True)
    put(table.s0w, t.get("s0w"))
    put(table.s0v, t.get("s0v"), cols=True)
    put(table.s1w, t.get("s1w"))
    put(table.s1v, t.get("s1v"), cols=True)


# ---------------------------------------------------------------------------
# reference layout: vocab_block_{i} [V // N + 1, K + 1], id g -> block g % N, row g // N
# ---------------------------------------------------------------------------
def export_reference_blocks(ckpt_dir: str, out_dir: str, block_num: int, *, with_slots: bool = True) -> list[str]:
    """Write ``vocab_block_{i}.npy`` (+ ``vocab_block_{i}_Adagrad.npy``) in the reference's layout."""
    meta = read_meta(ckpt_dir)
    V, K = meta["vocabulary_size"], meta["factor_num"]
    rows_per_block = V // block_num + 1
    os.makedirs(out_dir, exist_ok=True)
    blocks, slots = [], []
    for i in range(block_num):
        blocks.append(np.lib.format.open_memmap(os.path.join(out_dir, f"vocab_block_{i}.npy"), mode="w+",
                                                dtype=np.float32, shape=(rows_per_block, K + 1)))
        if with_slots:
            slots.append(np.lib.format.open_memmap(os.path.join(out_dir, f"vocab_block_{i}_Adagrad.npy"),
                                                   mode="w+", dtype=np.float32, shape=(rows_per_block, K + 1)))
    for s_rank, s_world, path in _iter_shards(ckpt_dir):
        for r0, t in _iter_row_chunks(path):
            n = t["w"].shape[0]
            gid = np.arange(r0, r0 + n, dtype=np.int64) * s_world + s_rank
            ok = gid < V
            gid = gid[ok]
            ref = np.concatenate([t["w"].float().numpy()[ok, None], t["v"].float().numpy()[ok]], axis=1)
            acc = np.concatenate([t["s0w"].numpy()[ok, None], t["s0v"].numpy()[ok]], axis=1)
            b, r = gid % block_num, gid // block_num
            for i in range(block_num):
                m = b == i
                blocks[i][r[m]] = ref[m]
                if with_slots:
                    slots[i][r[m]] = acc[m]
    files = []
    for i, arr in enumerate(blocks):
        arr.flush()
        files.append(os.path.join(out_dir, f"vocab_block_{i}.npy"))
    for arr in slots:
        arr.flush()
    with open(os.path.join(out_dir, "global_step.json"), "w") as f:
        json.dump({"global_step": meta["global_step"], "vocabulary_size": V, "factor_num": K,
                   "vocabulary_block_num": block_num}, f)
    return files


def import_reference_blocks(model, in_dir: str, block_num: int) -> None:
    """Load ``vocab_block_{i}.npy`` (reference layout) into the model's local table shard."""
    table = model.table
    gids = table.global_ids().cpu()
    ok = gids < table.vocab_size
    gids = gids[ok]
    local = torch.nonzero(ok).flatten()
    b, r = gids % block_num, torch.div(gids, block_num, rounding_mode="floor")
    for i in range(block_num):
        arr = np.load(os.path.join(in_dir, f"vocab_block_{i}.npy"), mmap_mode="r", allow_pickle=False)
        sp = os.path.join(in_dir, f"vocab_block_{i}_Adagrad.npy")
        acc = np.load(sp, mmap_mode="r", allow_pickle=False) if os.path.exists(sp) else None
        m = b == i
        if not bool(m.any()):
            continue
        rows = r[m].numpy()
        ref = torch.from_numpy(np.ascontiguousarray(arr[rows]))
        a = torch.from_numpy(np.ascontiguousarray(acc[rows])) if acc is not None else None
        table.load_reference_rows(local[m].to(table.device), ref, a)


# ---------------------------------------------------------------------------
# TensorFlow checkpoint (tensor bundle) in the reference's variable layout
# ---------------------------------------------------------------------------
def export_tf_checkpoint(ckpt_dir: str, out_dir: str, block_num: int, *, with_slots: bool = True) -> str:
    """Write ``out_dir/model.ckpt-<step>.{index,data-00000-of-00001}`` + ``checkpoint`` with the
    reference's variables: ``vocab_block_{i}`` [V//N+1, K+1] (col 0 = w), ``vocab_block_{i}/Adagrad``
    and ``global_step`` (what tf.train.Saver wrote for the reference, fm_model.py:269-284, :365)."""
    from .tf_bundle import write_bundle, write_checkpoint_state

    meta = read_meta(ckpt_dir)
    tmp = os.path.join(out_dir, ".blocks")
    export_reference_blocks(ckpt_dir, tmp, block_num, with_slots=with_slots)
    tensors = {"global_step": np.array(meta["global_step"], dtype=np.int64)}
    for i in range(block_num):
        tensors[f"vocab_block_{i}"] = np.load(os.path.join(tmp, f"vocab_block_{i}.npy"), mmap_mode="r")
        if with_slots:
            tensors[f"vocab_block_{i}/Adagrad"] = np.load(os.path.join(tmp, f"vocab_block_{i}_Adagrad.npy"),
                                                          mmap_mode="r")
    name = f"model.ckpt-{meta['global_step']}"
    write_bundle(os.path.join(out_dir, name), tensors)
    write_checkpoint_state(out_dir, name)
    shutil.rmtree(tmp, ignore_errors=True)
    return os.path.join(out_dir, name)


def import_tf_checkpoint(model, prefix: str, block_num: int | None = None) -> int:
    """Load a reference-layout TF checkpoint (``prefix`` = .../model.ckpt-N) into the model's
    local table shard; returns its global_step."""
    from .tf_bundle import read_bundle

    t = read_bundle(prefix)
    if block_num is None:
        block_num = sum(1 for k in t if k.startswith("vocab_block_") and "/" not in k)
    table = model.table
    gids = table.global_ids().cpu()
    ok = gids < table.vocab_size
    gids = gids[ok]
    local = torch.nonzero(ok).flatten()
    b, r = gids % block_num, torch.div(gids, block_num, rounding_mode="floor")
    for i in range(block_num):
        m = b == i
        if not bool(m.any()):
            continue
        rows = r[m].numpy()
        ref = torch.from_numpy(np.ascontiguousarray(t[f"vocab_block_{i}"][rows]))
        acc = t.get(f"vocab_block_{i}/Adagrad")
        a = torch.from_numpy(np.ascontiguousarray(acc[rows])) if acc is not None else None
        table.load_reference_rows(local[m].to(table.device), ref, a)
    step = int(t.get("global_step", np.array(0)))
    model.global_step = step
    if hasattr(model, "sr_reset"):
        model.sr_reset()
    return step
