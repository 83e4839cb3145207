"""Text input pipeline: files -> shuffled lines -> parsed CSR batches -> device.

Reference pipeline (tffm/fm_model.py:34-126), per ``shuffle_threads`` thread:
``string_input_producer(train_files, num_epochs, shuffle=True)`` ->
``TextLineReader.read_up_to(B)`` -> ``shuffle_batch(capacity = 4.5 B,
min_after_dequeue = 3 B, allow_smaller_final_batch)`` -> FmParser -> unique ->
``FIFOQueue(queue_size)``; weight files are read by a second file queue with the
same seed so that weight lines stay aligned with data lines.

Here:
* file order is reshuffled every epoch with a seeded RNG (same order for data
  and weight files, which are paired by index so alignment is exact);
* lines pass through a shuffle window of ``capacity = 4.5 B`` lines from which
  batches of B are drawn once ``min_after_dequeue + B`` are buffered (the
  final, smaller batch is emitted like ``allow_smaller_final_batch``);
* parsing runs in the native multi-threaded parser (``_fm_cpu``) with the GIL
  released; ``shuffle_threads`` producer threads feed a bounded queue
  (``queue_size`` batches) and a pinned-memory host->device copy runs ahead on
  a side stream, so parsing and H2D overlap the GPU step;
* multi-rank: each rank reads a disjoint subset of the files (rank::world, the
  reference's "each worker will retrieve one whole file", sample.cfg:68), or
  every world-th line when there are fewer files than ranks.
"""

from __future__ import annotations

import queue
import random
import threading
import weakref
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import native
from .batch import Batch


@dataclass
class ReaderState:
    epoch: int = 0
    batches_in_epoch: int = 0


def _read_lines(path: str) -> list[bytes]:
    with open(path, "rb") as f:
        return f.read().splitlines()


def parse_lines_to_batch(lines: list[bytes], vocab_size: int, hash_feature_id: bool, threads: int = 1,
                         weights: np.ndarray | None = None) -> Batch:
    labels, sizes, ids, vals = native.cpu().parse_lines(lines, int(vocab_size), bool(hash_feature_id), int(threads))
    return Batch.from_parsed(labels, sizes, ids, vals, weights)


def _load_bin_batch(files: list[str], vocab_size: int, hash_feature_id: bool) -> Batch:
    """All examples of binary CSR caches (in order) as one host batch."""
    from .device_cache import F_HASHED, read_header

    labels, weights, sizes, ids, vals = [], [], [], [], []
    hs = [read_header(f) for f in files]
    any_w = any(h["weights"] >= 0 for h in hs)
    for f, h in zip(files, hs):
        if h["vocab_size"] != vocab_size or bool(h["flags"] & F_HASHED) != bool(hash_feature_id):
            raise ValueError(f"{f}: converted with vocabulary_size {h['vocab_size']}, hash_feature_id "
                             f"{bool(h['flags'] & F_HASHED)}; the model uses {vocab_size}, {bool(hash_feature_id)}")
        mm = np.memmap(f, dtype=np.uint8, mode="r")
        n, z = h["n"], h["nnz"]
        labels.append(np.frombuffer(mm, np.float32, n, h["labels"]).copy())
        weights.append(np.frombuffer(mm, np.float32, n, h["weights"]).copy() if h["weights"] >= 0
                       else np.ones(n, np.float32))
        sizes.append(np.diff(np.frombuffer(mm, np.int64, n + 1, h["offsets"])).astype(np.int32))
        fid = np.frombuffer(mm, np.int32, z, h["ids"]).copy()
        if z and (int(fid.min()) < 0 or int(fid.max()) >= vocab_size):
            raise ValueError(f"{f}: feature ids outside [0, {vocab_size})")
        ids.append(fid)
        vals.append(np.frombuffer(mm, np.float32, z, h["vals"]).copy() if h["vals"] >= 0 else np.ones(z, np.float32))
        del mm
    cat = (lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt))
    return Batch.from_parsed(cat(labels, np.float32), cat(sizes, np.int32), cat(ids, np.int32),
                             cat(vals, np.float32), cat(weights, np.float32) if any_w else None)


def load_file_batch(files: list[str], weight_files: list[str] | None, vocab_size: int, hash_feature_id: bool,
                    threads: int = 4) -> Batch:
    """All lines of ``files`` (in order) as one batch (validation / predict); binary CSR
    caches (.fmb) are read directly (their weights are inside: no weight files)."""
    kinds = {bool(native.cpu().is_bin_file(f)) for f in files}
    if kinds == {True}:
        if weight_files:
            raise ValueError("binary CSR caches (.fmb) already hold the weights of their conversion; "
                             "remove the weight files")
        return _load_bin_batch(files, vocab_size, hash_feature_id)
    if len(kinds) > 1:
        raise ValueError("files mix binary CSR caches (.fmb) and text files")
    lines: list[bytes] = []
    for f in files:
        lines.extend(_read_lines(f))
    w = None
    if weight_files:
        wl: list[bytes] = []
        for f in weight_files:
            wl.extend(_read_lines(f))
        if len(wl) != len(lines):
            raise ValueError("weight files have %d lines, data files %d" % (len(wl), len(lines)))
        w = native.cpu().parse_floats(wl)
    return parse_lines_to_batch(lines, vocab_size, hash_feature_id, threads, w)


class TextBatchReader:
    """Iterator over shuffled, parsed training batches (host tensors)."""

    def __init__(self, files: list[str], weight_files: list[str] | None, batch_size: int, *, vocab_size: int,
                 hash_feature_id: bool = False, num_epochs: int = 1, shuffle: bool = True, seed: int = 0,
                 parse_threads: int = 4, rank: int = 0, world: int = 1, state: ReaderState | None = None):
        if weight_files and len(weight_files) != len(files):
            raise ValueError("The numbers of train files and weight files do not match.")
        if any(native.cpu().is_bin_file(f) for f in files):
            raise ValueError("binary CSR caches (.fmb) need the native loader ([Train] loader = native)")
        self.files = list(files)
        self.weight_files = list(weight_files) if weight_files else None
        self.B = int(batch_size)
        self.vocab_size = vocab_size
        self.hash = hash_feature_id
        self.num_epochs = num_epochs
        self.shuffle = shuffle
        self.seed = seed
        self.threads = parse_threads
        self.rank, self.world = rank, world
        self.state = state or ReaderState()
        self.capacity = int(3 * self.B + 1.5 * self.B)
        self.min_after = 3 * self.B
        self.fill = 0.0  # shuffle-window fill at the latest draw (-m "shuffle_queue")

    def window_fill(self) -> float:
        return self.fill

    def _my_files(self, epoch: int) -> list[tuple[str, str | None]]:
        pairs = list(zip(self.files, self.weight_files or [None] * len(self.files)))
        if self.shuffle:
            random.Random(self.seed * 1000003 + epoch).shuffle(pairs)
        if self.world > 1 and len(pairs) >= self.world:
            pairs = pairs[self.rank::self.world]
        return pairs

    def _lines(self, epoch: int):
        line_shard = self.world > 1 and len(self.files) < self.world
        for path, wpath in self._my_files(epoch):
            data = _read_lines(path)
            wl = _read_lines(wpath) if wpath else None
            if wl is not None and len(wl) != len(data):
                raise ValueError(f"{wpath}: {len(wl)} lines but {path} has {len(data)}")
            if line_shard:
                data = data[self.rank::self.world]
                wl = wl[self.rank::self.world] if wl is not None else None
            for i, ln in enumerate(data):
                if ln:
                    yield ln, (wl[i] if wl is not None else None)

    @staticmethod
    def _tag(b: Batch, epoch: int, count: int) -> Batch:
        # position AFTER this batch: what a checkpoint taken after consuming it must store
        b.reader_pos = (epoch, count)  # type: ignore[attr-defined]
        return b

    def _make(self, items) -> Batch:
        lines = [it[0] for it in items]
        w = None
        if self.weight_files:
            w = native.cpu().parse_floats([it[1] for it in items])
        return parse_lines_to_batch(lines, self.vocab_size, self.hash, self.threads, w)

    def __iter__(self):
        rng = random.Random(self.seed + 7919 * self.rank)
        skip = self.state.batches_in_epoch
        for epoch in range(self.state.epoch, self.num_epochs):
            self.state.epoch = epoch
            buf: list = []
            count = 0
            for item in self._lines(epoch):
                buf.append(item)
                if len(buf) >= self.capacity:
                    self.fill = len(buf) / self.capacity
                    if self.shuffle:
                        rng.shuffle(buf)
                    out, buf = buf[: self.B], buf[self.B:]
                    count += 1
                    if count > skip:
                        self.state.batches_in_epoch = count
                        yield self._tag(self._make(out), epoch, count)
            if self.shuffle:
                rng.shuffle(buf)
            while buf:
                self.fill = len(buf) / self.capacity
                out, buf = buf[: self.B], buf[self.B:]
                count += 1
                if count > skip:
                    self.state.batches_in_epoch = count
                    yield self._tag(self._make(out), epoch, count)
            skip = 0
            self.state.batches_in_epoch = 0
        self.state.epoch = self.num_epochs


class NativeTextReader:
    """The training-batch iterator backed by the native loader (csrc/cpu/loader.h).

    Same contract as ``TextBatchReader`` (epochs, per-epoch file shuffle, 4.5 B
    shuffle window, per-rank file / line sharding, weight-file pairing, exact
    resume from ``ReaderState``), but the whole host pipeline -- mmap'ed file
    reading, line splitting, the shuffle window, multi-threaded parsing and CSR
    assembly (int32 offsets and ids) -- runs in a C++ producer thread that
    keeps ``queue_size`` batches ready; Python only wraps the arrays.
    The batch composition (RNG streams) differs from ``TextBatchReader``.

    Binary CSR caches (``.fmb``, data/bincache.py) are detected by their magic: when every
    file is one, the loader copies pre-parsed examples instead of parsing text (same
    batches for the same seed; the weights come from the caches, so no weight files).
    ``device_cache`` (a GPU) uploads the caches to HBM once (data/device_cache.py) and
    the loader then ships only row numbers: batches are gathered on the device.
    """

    def __init__(self, files: list[str], weight_files: list[str] | None, batch_size: int, *, vocab_size: int,
                 hash_feature_id: bool = False, num_epochs: int = 1, shuffle: bool = True, seed: int = 0,
                 parse_threads: int = 4, rank: int = 0, world: int = 1, state: ReaderState | None = None,
                 queue_size: int = 4, gpu_parse: torch.device | str | None = None,
                 device_cache: torch.device | str | None = None, feed_device: torch.device | str | None = None):
        if weight_files and len(weight_files) != len(files):
            raise ValueError("The numbers of train files and weight files do not match.")
        kinds = {bool(native.cpu().is_bin_file(f)) for f in files}
        if len(kinds) > 1:
            raise ValueError("train files mix binary CSR caches (.fmb) and text files")
        self.binary = kinds == {True}
        if self.binary and weight_files:
            raise ValueError("binary CSR caches (.fmb) already hold the weights of their conversion; "
                             "remove weight_files")
        if self.binary:
            gpu_parse = None  # nothing to tokenize
        self.args = dict(files=list(files), weight_files=list(weight_files or []), batch_size=int(batch_size),
                         vocab_size=int(vocab_size), hash_feature_id=bool(hash_feature_id), shuffle=bool(shuffle),
                         num_epochs=int(num_epochs), seed=int(seed), threads=int(parse_threads), rank=int(rank),
                         world=int(world), queue_size=max(1, int(queue_size)))
        self.state = state or ReaderState()
        self.num_epochs = num_epochs
        self._loader = None
        # gpu_parse: the loader ships raw line bytes and the GPU tokenizer (hip/parse.hip) builds
        # the CSR on this device; yielded batches then live on the device, ready to use
        self.gpu = torch.device(gpu_parse) if gpu_parse is not None else None
        if self.gpu is not None and self.gpu.type != "cuda":
            self.gpu = None
        self.fallbacks = self.resizes = 0
        # feed_device (CPU parser, text files): the C++ feeder copies each parsed batch to this
        # device from its own thread, so batches come out on the device like the tokenizer's
        self.dds = None
        if device_cache is not None and self.binary and torch.device(device_cache).type == "cuda":
            from .device_cache import DeviceDataset

            self.dds = DeviceDataset(self.args["files"], device_cache, int(vocab_size), bool(hash_feature_id))
        # (binary caches assembled on the host take the feeder too: the loader's CSR rows are
        # copied to the device by the feeder thread, no Python producer thread)
        self.feed = None
        if feed_device is not None and self.gpu is None and self.dds is None:
            fd = torch.device(feed_device)
            self.feed = fd if fd.type == "cuda" else None

    def close(self) -> None:
        """Stop the native producer threads (feeder, loader); the iterator ends."""
        F = getattr(self, "_feeder", None)
        if F is not None:
            F.close()
        if self._loader is not None:
            self._loader.close()

    def queued(self) -> int:
        F = getattr(self, "_feeder", None)
        if F is not None:
            return int(F.queued())
        return self._loader.queued() if self._loader is not None else 0

    def window_fill(self) -> float:
        """Shuffle-window fill (0..1) at the loader's latest draw (-m "shuffle_queue")."""
        return float(self._loader.window_fill()) if self._loader is not None else 0.0

    def _estimate_slot_bytes(self) -> int:
        """Bytes of one batch slot: twice the batch's estimated text bytes (the longest average
        line over the heads of the files: files of one run can differ, e.g. with and without
        values)."""
        if getattr(self, "_slot_bytes", None) is None and self.binary:
            self._slot_bytes = 1  # (no text: the ids capacity comes from the caches' max_feats)
        if getattr(self, "_slot_bytes", None) is None:
            B = self.args["batch_size"]
            est = []
            for path in self.args["files"][:64]:
                try:
                    with open(path, "rb") as f:
                        head = f.read(1 << 20)
                    est.append(len(head) / max(1, head.count(b"\n")))
                except OSError:
                    pass
            avg = max(16.0, max(est)) if est else 256.0
            self._slot_bytes = int(B * avg * 2.0) + 4096
        return self._slot_bytes

    def _raw_slots(self) -> list[list[int]]:
        """Page-locked output slots of the loader's raw mode (GPU tokenizer): batches are assembled
        straight into them, so the host-to-device copy needs no staging copy.  queue_size + 3
        slots (queued batches, the one being copied / parsed, the one being finished, one spare)
        of ``_estimate_slot_bytes``; a larger batch falls back to a heap buffer (and, with the
        feeder, to the CPU parser)."""
        if getattr(self, "_slots", None) is None:
            B = self.args["batch_size"]
            nb, nl = self._estimate_slot_bytes(), B + 1
            self._slots = [(torch.empty(nb, dtype=torch.uint8, pin_memory=True),
                            torch.empty(nl, dtype=torch.int64, pin_memory=True),
                            torch.empty(B, dtype=torch.float32, pin_memory=True))
                           for _ in range(self.args["queue_size"] + 3)]
        return [[b.data_ptr(), b.numel(), ls.data_ptr(), ls.numel(), w.data_ptr(), w.numel()]
                for b, ls, w in self._slots]

    @property
    def inline(self) -> bool:
        """Batches come out complete and on the device (GPU tokenizer or CPU parser, fed by the C++
        feeder thread): a consumer needs no producer thread of its own (``Prefetcher`` iterates
        inline)."""
        return (self.gpu is not None or self.feed is not None) and _feeder_available()

    def __iter__(self):
        if self.inline:
            yield from self._iter_feeder()
            return
        slots = self._raw_slots() if self.gpu is not None else []
        L = native.cpu().TextLoader(start_epoch=self.state.epoch, skip_batches=self.state.batches_in_epoch,
                                    raw=self.gpu is not None, binary=self.binary, rows=self.dds is not None,
                                    raw_slots=slots, **self.args)
        self._loader = L
        dev = self.gpu if self.gpu is not None else (self.dds.device if self.dds is not None else None)
        stream = torch.cuda.Stream(dev) if dev is not None else None
        pending = None  # GPU tokenizer: batch k is launched, then k-1 finished and yielded
        try:
            while True:
                item = L.next()
                if item is None:
                    break
                if self.dds is not None:
                    rows, offsets, has_vals, max_feats, epoch, count = item
                    b = self._gather_batch(rows, offsets, has_vals, int(max_feats), stream)
                    self.state.epoch, self.state.batches_in_epoch = int(epoch), int(count)
                    b.reader_pos = (int(epoch), int(count))
                    yield b
                    continue
                if self.gpu is not None:
                    launched = self._gpu_launch(item, stream)
                    if pending is not None:
                        yield self._gpu_finish(pending)
                    pending = launched
                    continue
                labels, offsets, ids, vals, weights, max_feats, epoch, count = item
                b = Batch(torch.from_numpy(labels), torch.from_numpy(offsets), torch.from_numpy(ids),
                          None if vals is None else torch.from_numpy(vals),
                          None if weights is None else torch.from_numpy(weights), int(offsets[-1]),
                          max_feats=int(max_feats))
                self.state.epoch, self.state.batches_in_epoch = int(epoch), int(count)
                b.reader_pos = (int(epoch), int(count))
                yield b
            if pending is not None:
                yield self._gpu_finish(pending)
                pending = None
            self.state.epoch, self.state.batches_in_epoch = self.num_epochs, 0
        finally:
            L.close()

    # ------------------------------------------------------------------ C++ feeder (GPU tokenizer)
    def _device_slot(self) -> dict:
        """Device buffers of one feeder slot: raw bytes / line starts / weights copied in, the
        tokenizer's CSR out (ids / values sized for the densest possible batch: a token takes >= 2
        bytes), its counts / status / scan workspace."""
        dev, B, nb = self._feed_dev, self.args["batch_size"], self._slot_bytes
        cap = _bin_slot_cap(self.args["files"], B) if self.binary else nb // 2 + B + 1
        if self.gpu is None:
            nb = 1  # (parse mode: no raw bytes on the device)
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        return dict(bytes=torch.empty(nb, dtype=torch.uint8, device=dev),
                    ls=torch.empty(B + 1, dtype=torch.int64, device=dev), weights=torch.empty(B, **f32),
                    labels=torch.empty(B, **f32), offsets=torch.empty(B + 1, **i32), counts=torch.empty(B + 1, **i32),
                    ids=torch.empty(cap, **i32), vals=torch.empty(cap, **f32), status=torch.empty(8, **i32),
                    ws=torch.empty(max(1, int(native.hip().parse_workspace_bytes(B))), dtype=torch.uint8, device=dev))

    @staticmethod
    def _slot_ptrs(t: dict) -> list[int]:
        return [t["bytes"].data_ptr(), t["bytes"].numel(), t["ls"].data_ptr(), t["ls"].numel(), t["weights"].data_ptr(),
                t["labels"].data_ptr(), t["offsets"].data_ptr(), t["counts"].data_ptr(), t["ids"].data_ptr(),
                t["ids"].numel(), t["vals"].data_ptr(), t["status"].data_ptr(), t["ws"].data_ptr(), t["ws"].numel()]

    def _iter_feeder(self):
        """GPU-tokenizer batches from the C++ feeder (hip/feeder.hip): its thread takes the loader's
        raw batches (page-locked slots), copies them to a free device slot, launches the tokenizer,
        waits for it (CPU parse of a batch the GPU subset declines) and queues the finished batch;
        this generator only wraps the slot's tensors.  A device slot is handed back when the batch
        object dies: the feeder's stream then waits for the work queued so far on the releasing
        thread's current stream (the step that read it) before overwriting the slot."""
        raw = self.gpu is not None  # else the loader's CPU parser, the feeder copies the CSR over
        slots = self._raw_slots() if raw else []
        self._estimate_slot_bytes()
        L = native.cpu().TextLoader(start_epoch=self.state.epoch, skip_batches=self.state.batches_in_epoch,
                                    raw=raw, binary=self.binary, rows=False, raw_slots=slots, **self.args)
        self._loader = L
        dev = self.gpu if raw else self.feed
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self._feed_dev = dev
        F = native.hip().GpuTextFeeder(L.c_api(), dev.index, self.args["vocab_size"], self.args["hash_feature_id"])
        dslots = []

        def add_slot():
            with torch.cuda.device(dev):
                t = self._device_slot()
            torch.cuda.synchronize(dev)  # (allocation-time work done before the feeder's stream uses it)
            dslots.append(t)
            F.add_slot(self._slot_ptrs(t))

        for _ in range(max(6, self.args["queue_size"] + 4)):
            add_slot()
        F.start()
        self._feeder = F
        try:
            while True:
                r = F.next(100)
                if r is None:
                    break
                if isinstance(r, int):
                    # every slot is held by the consumer (e.g. list(reader)) while the feeder waits for one
                    if r == -1 and len(dslots) < 256:
                        add_slot()
                    continue
                if r[0] == "error":
                    raise (native.cpu().ParseError if r[1] else RuntimeError)(r[2])
                if r[0] == "resize":  # a batch denser than the slot estimate: larger ids / vals
                    _, d, need = r
                    cap = int(need * 1.25) + 1024
                    torch.cuda.synchronize(dev)  # (the steps that read the slot's old buffers have run)
                    with torch.cuda.device(dev):
                        dslots[d] = dict(dslots[d], ids=torch.empty(cap, dtype=torch.int32, device=dev),
                                         vals=torch.empty(cap, dtype=torch.float32, device=dev))
                    torch.cuda.synchronize(dev)
                    F.resize_ids(d, dslots[d]["ids"].data_ptr(), dslots[d]["vals"].data_ptr(), cap)
                    continue
                d, n, nnz, mf, has_vals, weighted, epoch, count = r
                t = dslots[d]
                b = Batch(t["labels"][:n], t["offsets"][: n + 1], t["ids"][:nnz], t["vals"][:nnz] if has_vals else None,
                          t["weights"][:n] if weighted else None, nnz, max_feats=mf)
                weakref.finalize(b, _feeder_release, F, d, dev)
                self.state.epoch, self.state.batches_in_epoch = int(epoch), int(count)
                b.reader_pos = (int(epoch), int(count))
                yield b
            self.state.epoch, self.state.batches_in_epoch = self.num_epochs, 0
        finally:
            self.fallbacks, self.resizes = int(F.fallbacks()), int(F.resizes())
            F.close()
            L.close()

    def _gather_batch(self, rows: np.ndarray, offsets: np.ndarray, has_vals: bool, max_feats: int, stream) -> Batch:
        """H2D of the batch's row numbers + offsets and the device gather (hip/batch_gather.hip)
        on ``stream``; returns a device batch whose work has completed."""
        dev = self.dds.device
        with torch.cuda.stream(stream):
            hr = torch.from_numpy(rows).pin_memory()
            ho = torch.from_numpy(offsets)
            d_rows = hr.to(dev, non_blocking=True)
            d_off = ho.pin_memory().to(dev, non_blocking=True)
            nnz = int(offsets[-1])
            labels, ids, vals, weights = self.dds.gather(d_rows, d_off, nnz, bool(has_vals), stream)
            stream.synchronize()
        return Batch(labels, d_off, ids, vals, weights, nnz, max_feats=max_feats, offsets_host=ho)

    def _stage(self, buf: np.ndarray, line_start: np.ndarray) -> tuple[torch.Tensor, torch.Tensor]:
        """Copy the raw batch into a reusable pinned staging slot (ring of 2, grown on demand).

        ``pin_memory()`` per batch allocated and filled a fresh page-locked buffer every time;
        the slots are allocated once and filled by torch's (multi-threaded) host copy.  A slot
        is reused two batches later, after ``_gpu_finish`` has waited for that batch's parse
        (which follows its host-to-device copy on the same stream)."""
        ring = getattr(self, "_ring", None)
        if ring is None:
            ring = self._ring = {"k": 0, "bytes": [None, None], "ls": [None, None]}
        k = ring["k"] = ring["k"] ^ 1
        n, m = buf.shape[0], line_start.shape[0]
        if ring["bytes"][k] is None or ring["bytes"][k].numel() < n:
            ring["bytes"][k] = torch.empty(max(n, int(1.25 * n)), dtype=torch.uint8, pin_memory=True)
        if ring["ls"][k] is None or ring["ls"][k].numel() < m:
            ring["ls"][k] = torch.empty(max(m, int(1.25 * m)), dtype=torch.int64, pin_memory=True)
        hb, hl = ring["bytes"][k][:n], ring["ls"][k][:m]
        hb.copy_(torch.from_numpy(buf))
        hl.copy_(torch.from_numpy(line_start))
        return hb, hl

    def _gpu_launch(self, item, stream):
        """Copy the raw lines of a loader item to the device (from its page-locked slot, or staged
        there first when the batch did not fit one) and launch the GPU tokenizer on ``stream`` --
        without waiting: the host takes the next batch while this one is copied and parsed
        (``_gpu_finish`` collects it and returns the slot to the loader)."""
        from ..ops import kernels as K

        slot = None
        if isinstance(item[0], int):  # (slot, nbytes, nlines, weights, epoch, count)
            slot, nbytes, nlines, weights, epoch, count = item
            hb, hl = self._slots[slot][0][:nbytes], self._slots[slot][1][: nlines + 1]
            buf = hb.numpy()
        else:
            buf, line_start, weights, epoch, count = item
        dev = self.gpu
        with torch.cuda.stream(stream):
            if slot is None:
                hb, hl = self._stage(buf, line_start)
            db = hb.to(dev, non_blocking=True)
            dl = hl.to(dev, non_blocking=True)
            # the weights' copy is queued BEFORE the tokenizer launch: parse_gpu_start records the
            # event that _gpu_finish waits on, so the event covers this copy too (a copy queued
            # after it could still be in flight when the compute stream reads b.weights).  The
            # source is page-locked (the caching host allocator keeps it alive until the copy ran)
            w = (None if weights is None
                 else torch.from_numpy(np.ascontiguousarray(weights)).pin_memory().to(dev, non_blocking=True))
            pp = K.parse_gpu_start(db, dl, self.args["vocab_size"], self.args["hash_feature_id"], stream=stream)
        return pp, buf, w, int(epoch), int(count), slot

    def _gpu_finish(self, launched) -> Batch:
        """Wait for a launched tokenizer pass and wrap its outputs (CPU parser when the batch has
        syntax outside the GPU subset or errors); the returned device batch is complete."""
        pp, buf, w, epoch, count, slot = launched
        pg = pp.finish()
        dev = self.gpu
        if pg.fallback:
            self.fallbacks += 1
            labels, sizes, ids, vals = native.cpu().parse_buffer(buf, self.args["vocab_size"],
                                                                 self.args["hash_feature_id"],
                                                                 self.args["threads"])
            b = Batch.from_parsed(labels, sizes, ids, vals).to(dev)
            b.weights = w
            torch.cuda.current_stream(dev).synchronize()
        else:
            b = Batch(pg.labels, pg.offsets, pg.ids, pg.vals, w, pg.nnz, max_feats=pg.max_feats)
        if slot is not None:  # its copy and parse are complete (finish synchronised them)
            self._loader.release(slot)
        self.state.epoch, self.state.batches_in_epoch = epoch, count
        b.reader_pos = (epoch, count)
        return b


def _bin_slot_cap(files: list[str], B: int) -> int:
    """ids / vals entries of a feeder slot for .fmb caches (csrc/cpu/bincsr.h header: i64 n at byte
    16, i64 nnz at 24, i32 max_feats at 40): the caches' mean features per example x B with 50%
    headroom, at most B x their largest example; a denser batch gets larger buffers through the
    feeder's resize request (next() -> "resize")."""
    import struct

    n = nnz = 0
    mf = 1
    for f in files:
        with open(f, "rb") as fh:
            head = fh.read(64)
        fn, fnnz = struct.unpack_from("<qq", head, 16)
        n, nnz = n + fn, nnz + fnnz
        mf = max(mf, struct.unpack_from("<i", head, 40)[0])
    mean = nnz / max(n, 1)
    return min(B * mf, int(B * mean * 1.5) + 4096) + 1


def _feeder_available() -> bool:
    try:
        return hasattr(native.hip(), "GpuTextFeeder")
    except Exception:  # noqa: BLE001  (no HIP module: the Python-driven GPU tokenizer path)
        return False


def _feeder_release(F, d: int, dev: torch.device) -> None:
    try:
        F.release(d, torch.cuda.current_stream(dev).cuda_stream)
    except Exception:  # noqa: BLE001  (interpreter shutdown / feeder closed: nothing to hand back)
        pass


class Prefetcher:
    """Background producer threads + bounded queue + pinned H2D on a side stream.

    ``queue_size`` mirrors the reference's example FIFOQueue capacity; ``size()``
    is what ``-m`` reports as ``example_queue`` fill.
    """

    _END = object()

    def __init__(self, reader: TextBatchReader, device: torch.device, queue_size: int = 8):
        self.reader = reader
        self.device = torch.device(device)
        self.q: queue.Queue = queue.Queue(maxsize=max(1, queue_size))
        self.queue_size = max(1, queue_size)
        self._err: BaseException | None = None
        self._stop = threading.Event()
        # a reader whose batches come out complete on the device from a native producer thread
        # (NativeTextReader + C++ feeder) is iterated inline: no Python thread, no queue hop
        self.inline = bool(getattr(reader, "inline", False))
        self._stream = None
        if self.inline:
            return
        self._th = threading.Thread(target=self._run, name="fm-reader", daemon=True)
        self._stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._th.start()

    def _run(self):
        try:
            for b in self.reader:
                if self._stop.is_set():
                    return
                if b.ids.device.type == "cuda":
                    self.q.put((b, "device", None))   # tokenized on the GPU, already complete
                elif self._stream is not None:
                    b = b.pin_memory()
                    with torch.cuda.stream(self._stream):
                        db = b.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self._stream)
                    self.q.put((db, ev, b))
                else:
                    self.q.put((b, None, None))
        except BaseException as e:  # noqa: BLE001
            self._err = e
        finally:
            self.q.put((self._END, None, None))

    def size(self) -> int:
        if self.inline:
            return min(self.queue_size, int(self.reader.queued()))
        return self.q.qsize()

    def shuffle_fill(self) -> float:
        """The reader's shuffle-window fill (0..1), the reference's shuffle_queue metric."""
        f = getattr(self.reader, "window_fill", None)
        return float(f()) if f is not None else 0.0

    def __iter__(self):
        if self.inline:
            yield from self.reader
            return
        while True:
            item, ev, _host = self.q.get()
            if item is self._END:
                if self._err is not None:
                    raise self._err
                return
            if ev == "device":
                # produced on the reader's stream (synchronised): the compute stream uses it from now on
                cur = torch.cuda.current_stream(self.device)
                for t in (item.labels, item.offsets, item.ids, item.vals, item.weights):
                    if t is not None:
                        t.record_stream(cur)
            elif ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                # the batch was allocated on the side stream: tell the caching allocator
                # it is in use on the compute stream too
                for t in (item.labels, item.offsets, item.ids, item.vals, item.weights):
                    if t is not None:
                        t.record_stream(cur)
                # keep the pinned source alive until the copy has been consumed
                item._host_ref = _host  # type: ignore[attr-defined]
                item.ready = ev  # type: ignore[attr-defined]  # other streams (lookahead plans) wait on it
            yield item

    def close(self):
        self._stop.set()
        if self.inline and hasattr(self.reader, "close"):
            self.reader.close()
