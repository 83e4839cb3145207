"""Training / prediction drivers (the reference's run_tffm.py train() and predict()).

Reference behaviour kept (run_tffm.py:10-90, :213-231):
* ``========  train  ========`` banner; per step ``-- Global Step: %d; Avg loss: %.5f;``;
* ``-m``: ``speed: <ex/s> shuffle_queue: x% example_queue: y%`` per step;
* every ``save_steps``: validation loss ``validation loss at step %d: %.8f`` and
  early stop below ``tolerance`` ("Loss on validation data set is below
  tolerance. Training completed."), checkpoint (CheckpointSaverHook);
* automatic restore of the latest checkpoint in ``log_dir`` (MonitoredTrainingSession);
* end: ``Average speed:  <ex/s>  ex/s`` and ``Model saved to  <log_dir>``;
* ``-t FILE``: chrome-trace timeline (reference: first step only; here the
  first few steps after one warm-up step);
* predict: ``<predict_file>_score`` with one raw score (logit) per line.

Multi-rank runs are synchronous: every step all ranks agree (one tiny
all-reduce) that each still has a batch, so the run ends cleanly when the first
rank's data is exhausted (the reference's OutOfRangeError, run_tffm.py:43-44).
"""

from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

from .config import FMRunConfig
from .utils.fault import maybe_inject
from .utils.trace import roctx_range
from .data.reader import NativeTextReader, Prefetcher, ReaderState, TextBatchReader, load_file_batch
from .models.fm import FactorizationMachine
from .ops.kernels import check_device_errors
from .parallel.dist import DistContext
from .utils import checkpoint as ckpt
from .utils.metrics import MetricsLogger


def _resolve_device(cfg: FMRunConfig, ctx: DistContext | None) -> torch.device:
    if ctx is not None and ctx.world > 1:
        return ctx.device
    if cfg.device in ("cpu", "cuda"):
        return torch.device("cuda" if cfg.device == "cuda" else "cpu")
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


# Version of the loader's shuffle draws (csrc/cpu/loader.cpp ``bounded``): 1 = ``rng() % range``
# (round 2), 2 = multiply-high.  Stored with every reader position; a resume across versions warns.
DRAW_VERSION = 2


class Trainer:
    def __init__(self, cfg: FMRunConfig, ctx: DistContext | None = None, *, monitor: bool = False,
                 trace: str | None = None, printer=print, trace_steps: int = 5):
        self.cfg = cfg
        self.ctx = ctx
        self.world = ctx.world if ctx is not None else 1
        self.rank = ctx.rank if ctx is not None else 0
        self.monitor = monitor
        self.trace = trace
        self.trace_steps = trace_steps
        self.print = printer if self.rank == 0 else (lambda *a, **k: None)
        self.device = _resolve_device(cfg, ctx)
        self.model = FactorizationMachine(cfg.fm_config(), device=self.device,
                                          dist=ctx if self.world > 1 else None)
        self.reader_state = ReaderState()
        self.restored_from = None

    def close(self) -> None:
        """Release the model's executor resources (graphs, exchange, streams)."""
        self.model.close()

    def __enter__(self) -> "Trainer":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    # ------------------------------------------------------------------
    def restore(self) -> bool:
        path = ckpt.latest_checkpoint(self.cfg.log_dir)
        if path is None:
            return False
        meta = ckpt.restore_checkpoint(self.model, path)
        # this rank's own reader position (each rank reads its own file subset); a checkpoint
        # from another world size (or without per-rank entries) falls back to rank 0's
        per_rank = meta.get("reader_states") or {}
        if int(meta.get("reader_world", 1)) == self.world and str(self.rank) in per_rank:
            rs = per_rank[str(self.rank)] or {}
        else:
            rs = meta.get("reader_state") or {}
            if self.world > 1:
                self.print(f"Checkpoint reader positions are for world {meta.get('reader_world', 1)}; "
                           f"every rank resumes at rank 0's position")
        self.reader_state = ReaderState(epoch=int(rs.get("epoch", 0)),
                                        batches_in_epoch=int(rs.get("batches_in_epoch", 0)))
        dv = rs.get("draw_version") if rs else None
        if rs and dv is None:
            # (checkpoints written before the field existed: the draws may or may not be this build's)
            self.print(f"Note: checkpoint reader position does not record its shuffle draw version; resuming "
                       f"with this build's draws (version {DRAW_VERSION})")
        elif rs and int(dv) != DRAW_VERSION:
            # the loader's shuffle draws changed between the builds: the same seed gives another line
            # order, so replaying batches_in_epoch batches does not land on the same examples
            self.print(f"Warning: checkpoint reader position was written with shuffle draw version "
                       f"{dv} (this build: {DRAW_VERSION}); the resumed epoch repeats or skips some examples")
        self.restored_from = path
        self.print(f"Restored checkpoint {path} (global step {self.model.global_step})")
        return True

    def save(self) -> str | None:
        if not self.cfg.log_dir:
            return None
        rs = {"epoch": self.reader_state.epoch, "batches_in_epoch": self.reader_state.batches_in_epoch,
              "draw_version": DRAW_VERSION}
        return ckpt.save_checkpoint(self.model, self.cfg.log_dir, self.model.global_step, reader_state=rs,
                                    ctx=self.ctx if self.world > 1 else None)

    def _all_have_batch(self, have: bool) -> bool:
        if self.world == 1:
            return have
        t = torch.tensor([1 if have else 0], dtype=torch.int32, device=self.ctx.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.ctx.group)
        return bool(t.item())

    def _global_loss(self, loss_sum: float, n: int) -> float:
        if self.world == 1:
            return loss_sum / max(n, 1)
        t = torch.tensor([loss_sum, float(n)], dtype=torch.float64, device=self.ctx.device)
        dist.all_reduce(t, group=self.ctx.group)
        return float(t[0] / max(t[1], 1.0))

    # ------------------------------------------------------------------
    def load_validation(self):
        c = self.cfg
        if not c.validation_data_files:
            return None
        self.print("Preloading validation data...")
        b = load_file_batch(c.validation_data_files, c.validation_weight_files, c.vocabulary_size,
                            c.hash_feature_id, c.parse_threads)
        if self.world > 1:
            idx = torch.arange(self.rank, b.B, self.world)
            b = _take(b, idx)
        return b.to(self.device)

    def _device_cache(self):
        """The device to keep .fmb training files on, or None ([Train] device_cache)."""
        c = self.cfg
        if c.device_cache == "false" or self.device.type != "cuda" or not c.train_files:
            return None
        from .data import bincache, device_cache

        if not all(bincache.is_bin_file(f) for f in c.train_files):
            return None
        if c.device_cache == "auto":
            free, _ = torch.cuda.mem_get_info(self.device)
            if device_cache.dataset_bytes(c.train_files) > 0.4 * free:
                return None
        return self.device

    def validation_loss(self, vb) -> float:
        fo = self.model.forward(vb, loss=self.cfg.loss_type)
        return self._global_loss(float(fo.loss_sum), vb.B)

    # ------------------------------------------------------------------
    def train(self) -> dict:
        c = self.cfg
        self.restore()
        vb = self.load_validation()
        kw = dict(vocab_size=c.vocabulary_size, hash_feature_id=c.hash_feature_id, num_epochs=c.num_epochs,
                  shuffle=c.shuffle, seed=c.seed, parse_threads=c.parse_threads, rank=self.rank, world=self.world,
                  state=ReaderState(self.reader_state.epoch, self.reader_state.batches_in_epoch))
        if c.loader == "native":
            reader = NativeTextReader(c.train_files, c.weight_files or None, c.batch_size,
                                      gpu_parse=self.device if c.gpu_parse else None,
                                      feed_device=self.device if self.device.type == "cuda" else None,
                                      device_cache=self._device_cache(), **kw)
            if reader.dds is not None:
                self.print(f"Training data resident on {self.device}: {reader.dds.N} examples, "
                           f"{reader.dds.nbytes / 2**30:.2f} GiB")
        else:
            reader = TextBatchReader(c.train_files, c.weight_files or None, c.batch_size, **kw)
        pf = Prefetcher(reader, self.device, queue_size=max(1, min(c.queue_size, 64)))
        metrics = MetricsLogger(c.log_dir if self.rank == 0 else None, every=c.save_summaries_steps)
        self.print("========", "train", "========")
        st = time.time()
        start_step = self.model.global_step
        step_num = start_step
        it = iter(pf)
        prof = None
        ended_early = False
        last_loss = float("nan")

        def fetch():
            with roctx_range("input_wait"):
                try:
                    nb = next(it)
                except StopIteration:
                    nb = None
            return nb, self._all_have_batch(nb is not None)

        def report(p):
            """Print / log a finished step.  Called once the NEXT step is enqueued, so reading
            this step's loss (a host sync) overlaps the device work of the next one."""
            sn, o, t0 = p
            loss = o.mean_loss()  # the reference fetches the loss every step
            tend = time.time()
            if self.monitor:
                q = pf.size()
                self.print("speed:", c.batch_size * self.world / max(tend - t0, 1e-9),
                           "shuffle_queue: %.2f%%" % (100.0 * pf.shuffle_fill()),
                           "example_queue: %.2f%%" % (q * 100.0 / pf.queue_size))
            if c.log_steps <= 1 or sn % c.log_steps == 0:
                self.print("-- Global Step: %d; Avg loss: %.5f;" % (sn, loss))
            metrics.log(sn, loss=loss, exq_size=pf.size(), shuffle_fill=pf.shuffle_fill())
            return loss, tend

        batch, have = fetch()
        nxt, nhave = fetch() if have else (None, False)
        pending = None
        tprev = time.time()
        # steady state: from the end of the first epoch (input caches, page cache, lazy
        # kernel loads and allocator growth are warm by then) to the end of the run
        steady_t0, steady_step = None, None
        while have:
            # lookahead: the next two batches (when every rank has them) let the executors build
            # their dedup / id exchange / early row exchange while this step computes
            nxt2, nhave2 = fetch() if nhave else (None, False)
            if self.trace and prof is None and step_num == start_step + 1:
                prof = _start_profiler()
            with roctx_range("train_step"):
                out = self.model.train_step(batch, nxt if nhave else None, nxt2 if nhave2 else None)
            step_num = self.model.global_step
            if batch.reader_pos is not None:  # position of the last CONSUMED batch (the reader runs ahead)
                self.reader_state.epoch, self.reader_state.batches_in_epoch = batch.reader_pos
                if steady_t0 is None and batch.reader_pos[0] >= 1:
                    if self.device.type == "cuda":
                        torch.cuda.synchronize(self.device)
                    steady_t0, steady_step = time.time(), step_num - 1
            if pending is not None:
                last_loss, tprev = report(pending)
            pending = (step_num, out, tprev)
            if prof is not None and step_num >= start_step + 1 + self.trace_steps:
                _stop_profiler(prof, self.trace)
                prof = None
                self.trace = None
            if step_num % max(c.save_steps, 1) == 0:
                last_loss, tprev = report(pending)
                pending = None
                if vb is not None:
                    v_loss = self.validation_loss(vb)
                    self.print("validation loss at step %d: %.8f" % (step_num, v_loss))
                    metrics.log(step_num, force=True, validation_loss=v_loss)
                    if c.tolerance is not None and v_loss < c.tolerance:
                        self.print("Loss on validation data set is below tolerance. Training completed.")
                        ended_early = True
                check_device_errors(self.device)  # (kernels' sticky error word: fail before saving)
                if c.log_dir:
                    self.save()
            maybe_inject(step_num, self.rank)
            if ended_early or (c.max_steps is not None and step_num - start_step >= c.max_steps):
                break
            batch, have = nxt, nhave
            nxt, nhave = nxt2, nhave2
        if pending is not None:
            last_loss, _ = report(pending)
        if prof is not None:
            _stop_profiler(prof, self.trace)
        pf.close()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        check_device_errors(self.device)
        total = time.time() - st
        speed = (step_num - start_step) * c.batch_size * self.world / max(total, 1e-9)
        self.print("Average speed: ", speed, " ex/s")
        steady = None
        if steady_t0 is not None and step_num - steady_step > 0:
            steady = (step_num - steady_step) * c.batch_size * self.world / max(time.time() - steady_t0, 1e-9)
            self.print("Steady-state speed (epochs 2+): ", steady, " ex/s")
        if c.log_dir:
            self.save()
        self.print("Model saved to ", c.log_dir)
        metrics.close()
        return {"steps": step_num - start_step, "global_step": step_num, "avg_speed": speed, "steady_speed": steady,
                "last_loss": last_loss, "early_stop": ended_early}

    # ------------------------------------------------------------------
    def predict(self) -> list[str]:
        c = self.cfg
        if not self.restore():
            raise FileNotFoundError(f"no checkpoint found in {c.log_dir}")
        self.print("========", "predict", "========")
        written = []
        for path in c.predict_files:
            b = load_file_batch([path], None, c.vocabulary_size, c.hash_feature_id, c.parse_threads)
            if self.world > 1:
                idx = torch.arange(self.rank, b.B, self.world)
                mine = _take(b, idx).to(self.device)
                scores = self.model.predict(mine).cpu().numpy()
                parts = [None] * self.world
                dist.all_gather_object(parts, scores, group=self.ctx.cpu_group)
                full = np.empty(b.B, dtype=np.float32)
                for r, p in enumerate(parts):
                    full[r::self.world] = p
                scores = full
            else:
                scores = self.model.predict(b.to(self.device)).cpu().numpy()
            if self.rank == 0:
                out = path + "_score"
                with open(out, "w") as f:
                    for s in scores:
                        f.write(str(np.float32(s)) + "\n")
                written.append(out)
        self.print("Done. Scores saved to same directory as predict files")
        return written


def _take(b, idx: torch.Tensor):
    """Sub-batch of examples ``idx`` (host tensors)."""
    from .data.batch import Batch

    o = b.offsets.long()
    sizes = (o[1:] - o[:-1])[idx]
    starts = o[:-1][idx]
    # feature positions of the chosen examples, vectorised: start of each example repeated
    # over its features + the position inside the example
    ends = torch.cumsum(sizes, 0)
    total = int(ends[-1]) if idx.numel() else 0
    within = torch.arange(total, dtype=torch.long) - torch.repeat_interleave(ends - sizes, sizes)
    gather = torch.repeat_interleave(starts, sizes) + within
    offs = torch.zeros(idx.numel() + 1, dtype=torch.int32)
    offs[1:] = torch.cumsum(sizes, 0)
    return Batch(b.labels[idx], offs, b.ids[gather], None if b.vals is None else b.vals[gather],
                 None if b.weights is None else b.weights[idx], int(offs[-1]), max_feats=b.max_feats)


def _start_profiler():
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    prof = torch.profiler.profile(activities=acts)
    prof.__enter__()
    return prof


def _stop_profiler(prof, trace: str) -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    prof.__exit__(None, None, None)
    if not trace.endswith(".json"):
        trace += ".json"
    d = os.path.dirname(trace)
    if d:
        os.makedirs(d, exist_ok=True)
    prof.export_chrome_trace(trace)
