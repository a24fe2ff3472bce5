"""Phase ranges and timelines (SURVEY.md §5 "Tracing / profiling").

The reference has no tracing (only ``model.summary()`` prints).  Two layers here:

* :func:`trange` — a named range around a training phase (sample, critic W-terms, gradient
  penalty, optimizer, all-reduce, generator).  When ``HFREP_TRACE=1`` it pushes a ROCTX range
  (``librocprofiler-sdk-roctx.so``, else the legacy ``libroctx64.so``; visible with
  ``rocprofv3 --marker-trace --kernel-trace``) and a ``torch.profiler.record_function`` scope;
  otherwise it is a no-op (one flag check), so the trainer calls it unconditionally.  Ranges are
  host-side: inside a hipGraph capture they mark the capture, not the replays.
* :func:`profile_steps` — runs a callable for a few steps under ``torch.profiler`` (CPU + HIP
  activities) and exports a Chrome trace plus the per-kernel table.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_ENABLED = os.environ.get("HFREP_TRACE", "0") == "1"
_roctx = None
_roctx_tried = False


def enable(on: bool = True) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def _lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for cand in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                     "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(cand)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


@contextlib.contextmanager
def trange(name: str):
    if not _ENABLED:
        yield
        return
    import torch

    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if _ENABLED and _lib() is not None:
        _roctx.roctxMarkA(name.encode())


def profile_steps(step_fn, steps: int, out_path: str, row_limit: int = 30) -> str:
    """Run ``step_fn()`` ``steps`` times under torch.profiler; write ``out_path`` (Chrome trace JSON)
    and ``out_path + '.txt'`` (kernel table sorted by device time).  Returns the table."""
    import torch
    from torch.profiler import ProfilerActivity, profile

    gpu = torch.cuda.is_available()
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if gpu else [])
    prev = _ENABLED
    enable(True)
    try:
        with profile(activities=acts, record_shapes=False) as prof:
            for _ in range(steps):
                step_fn()
            if gpu:
                torch.cuda.synchronize()
    finally:
        enable(prev)
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    prof.export_chrome_trace(out_path)
    table = prof.key_averages().table(sort_by="cuda_time_total" if gpu else "cpu_time_total", row_limit=row_limit)
    with open(out_path + ".txt", "w") as fh:
        fh.write(table)
    return table
