"""Tracing: chrome-trace timelines of training steps.

Reference: ``-t FILE`` runs the FIRST step with FULL_TRACE RunOptions and writes
``timeline.Timeline(step_stats).generate_chrome_trace_format()`` to FILE(.json)
(run_tffm.py:33-37, :84-90).  Here ``-t`` records N steps after warm-up with
torch.profiler (CPU + ROCm/roctracer kernel activity) and exports a chrome
trace; kernel-level counters come from rocprofv3 (tools/profile.sh).
"""

from __future__ import annotations

import os
from typing import Callable

import torch


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
