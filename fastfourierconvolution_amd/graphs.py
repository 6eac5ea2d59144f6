"""hipGraph capture of a whole step, safe next to RCCL (one process per GPU).

A step of this package (generator forward, or the G + D train step) launches only library
kernels and, under SyncBN, RCCL all-reduces; it allocates nothing and never synchronises, so it
captures into one hipGraph.  Two rules make that capture safe when a ``nccl`` (RCCL) process
group exists:

* **capture in ``thread_local`` mode, after a device synchronise.**  ``ProcessGroupNCCL``'s
  watchdog thread polls the end events of every EAGER collective (the warm-up's SyncBN
  all-reduces) with ``hipEventQuery``.  Under the default ``global`` capture mode any other
  thread's "unsafe" call during a capture is an error: the watchdog then sees a HIP error and
  rethrows it (``TORCH_NCCL_RETHROW_CUDA_ERRORS`` defaults to on), which terminates the process
  with SIGABRT -- the one-off exit 134 of round 2 ("graph capture and the RCCL
  watchdog").  ``thread_local`` restricts only the capturing thread; the synchronise retires the
  eager work first, so the watchdog's queries find it complete.
  ``tools/capture_mode_probe.hip`` measures what HIP returns to a second thread in each mode.
* **agree before the first replay.**  Every rank must replay the same collectives.  The capture
  result is MIN-all-reduced right after capture ends and before any replay; a rank whose capture
  failed makes every rank time eagerly (replaying first would pair a graph's SyncBN
  all-reduces with the failing rank's int32 vote).
"""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist

__all__ = ["CAPTURE_MODE", "agree", "capture_step"]

CAPTURE_MODE = os.environ.get("FFC_CAPTURE_MODE", "thread_local")


def agree(ok: bool, group=None, device: torch.device | None = None) -> bool:
    """True iff ``ok`` on every rank of ``group`` (MIN all-reduce; a no-op without a group)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return ok
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _forced_failure() -> bool:
    """test hook: FFC_FAIL_CAPTURE_RANK=<r> makes rank r's capture fail (gloo tests, bench dry run)"""
    r = os.environ.get("FFC_FAIL_CAPTURE_RANK")
    return r is not None and int(r) == int(os.environ.get("RANK", "0"))


def capture_step(step, group=None, warmup: int = 1, capture=None):
    """Warm ``step`` up on a side stream, synchronise, capture it into a CUDAGraph (thread-local
    mode) and return the graph (``graph.ffc_output``: what the captured step returned, rewritten by
    every replay) -- or None on EVERY rank if any rank's capture failed.  ``capture``
    replaces the capture itself (``capture(step) -> graph``; CPU tests)."""
    graph, err = None, None
    try:
        if _forced_failure():
            raise RuntimeError("capture failure forced by FFC_FAIL_CAPTURE_RANK")
        if capture is not None:
            graph = capture(step)
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(max(0, warmup)):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                out = step()
            # the captured step's output tensors: every replay rewrites them in place (bench.py
            # checks the timed artifact itself against the oracle after the timed replays)
            g.ffc_output = out
            graph = g
    except Exception as e:          # capture unsupported here: the caller times eagerly
        err = e
        graph = None
    if not agree(graph is not None, group):
        if err is not None:
            print(f"[ffc] graph capture failed ({err}); running eagerly", file=sys.stderr)
        else:
            print("[ffc] graph capture failed on another rank; running eagerly", file=sys.stderr)
        return None
    return graph
