"""Failure detection hooks and an environment-driven fault injector.

The reference relies on TF's MonitoredTrainingSession to re-create a session
and restore the latest checkpoint after a PS/worker failure (SURVEY.md §5.3,
run_tffm.py:217-221).  Here recovery is torchrun's: ``--max-restarts N``
relaunches every rank and the trainer auto-resumes from the latest checkpoint
in ``log_dir`` (table, optimizer slots, global step and the reader position).
Hangs become errors through the process-group timeout with
TORCH_NCCL_ASYNC_ERROR_HANDLING=1 (parallel/dist.py).

Fault injection for the resume test (tests/test_fault_resume.py):
  FM_FAULT_STEP=s    kill the process right after global step s completed
  FM_FAULT_RANK=r    ... only on rank r (default 0)
  FM_FAULT_MARKER=f  fire only if file f does not exist yet (it is created),
                     so the restarted job runs through
  FM_FAULT_EXIT=c    exit code (default 17)
"""

from __future__ import annotations

import os
import sys


def maybe_inject(step: int, rank: int) -> None:
    s = os.environ.get("FM_FAULT_STEP")
    if not s or step != int(s) or rank != int(os.environ.get("FM_FAULT_RANK", "0")):
        return
    marker = os.environ.get("FM_FAULT_MARKER")
    if marker:
        if os.path.exists(marker):
            return
        with open(marker, "w") as f:
            f.write(str(step))
    print(f"[fault] injected failure after step {step} on rank {rank}", file=sys.stderr, flush=True)
    os._exit(int(os.environ.get("FM_FAULT_EXIT", "17")))
