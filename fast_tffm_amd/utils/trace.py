"""Tracing: chrome-trace timelines of training steps, and roctx ranges.

Reference: ``-t FILE`` runs the FIRST step with FULL_TRACE RunOptions and writes
``timeline.Timeline(step_stats).generate_chrome_trace_format()`` to FILE(.json)
(run_tffm.py:33-37, :84-90).  Here ``-t`` records N steps after warm-up with
torch.profiler (CPU + ROCm/roctracer kernel activity) and exports a chrome
trace; kernel-level counters come from rocprofv3 (tools/gpu_iter.sh, gpu_pmc.sh).

``roctx_range(name)`` marks host phases (parse wait, plan, gather, a2a, fwd,
bwd, update) for ``rocprofv3 --marker-trace`` when ``FM_ROCTX=1``; otherwise
it costs one dict lookup.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Callable

import torch

_ROCTX_ON = os.environ.get("FM_ROCTX", "0") == "1"
_roctx = None


def _roctx_lib():
    """rocprofiler-sdk's roctx (what rocprofv3 --marker-trace records), else torch's nvtx/roctx shim."""
    global _roctx
    if _roctx is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = (lambda s, _l=lib: _l.roctxRangePushA(s.encode()), lib.roctxRangePop)
                break
            except (OSError, AttributeError):
                continue
        else:
            _roctx = (torch.cuda.nvtx.range_push, torch.cuda.nvtx.range_pop)
    return _roctx


def set_roctx(on: bool) -> None:
    global _ROCTX_ON
    _ROCTX_ON = bool(on)


@contextlib.contextmanager
def roctx_range(name: str):
    if not _ROCTX_ON:
        yield
        return
    push, pop = _roctx_lib()
    push(name)
    try:
        yield
    finally:
        pop()


def profile_steps(step_fn: Callable[[int], object], n_steps: int, out_path: str) -> str:
    if not out_path.endswith(".json"):
        out_path += ".json"
    d = os.path.dirname(out_path)
    if d:
        os.makedirs(d, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        for i in range(n_steps):
            with torch.profiler.record_function(f"train_step_{i}"):
                step_fn(i)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    prof.export_chrome_trace(out_path)
    return out_path
