"""Loader for the in-tree gfx950 kernel library (``ops/_hfrep_native.so``).

Policy (so GPU runs can never pass on a silent PyTorch fallback):

* On a machine with a visible GPU the library MUST load; if it is missing or fails to load,
  :func:`native` raises.  Set ``HFREP_ALLOW_TORCH_FALLBACK=1`` to deliberately run the
  composed-PyTorch reference path on GPU (debug only; it is never the default).
* On a CPU-only machine the native ops are simply unavailable and the reference
  implementation in :mod:`hfrep.ops.reference` is used for CPU tensors.
"""
from __future__ import annotations

import os
import threading

import torch

# HFREP_NATIVE_LIB: an alternative build of the same library (A/B kernel experiments only)
_LIB_PATH = os.environ.get("HFREP_NATIVE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                               "_hfrep_native.so")
_lock = threading.Lock()
_loaded = None  # None = not tried, True/False afterwards
_err: Exception | None = None


def library_path() -> str:
    return _LIB_PATH


def _try_load() -> bool:
    global _loaded, _err
    with _lock:
        if _loaded is not None:
            return _loaded
        if not os.path.exists(_LIB_PATH):
            _err = FileNotFoundError(
                f"{_LIB_PATH} not built; run `python build_native.py` (or __graft_entry__.build())"
            )
            _loaded = False
            return False
        try:
            torch.ops.load_library(_LIB_PATH)
            _loaded = True
        except Exception as e:  # pragma: no cover - depends on the box
            _err = e
            _loaded = False
        return _loaded


def available() -> bool:
    """True when the kernel library is loaded (it only runs on GPU tensors)."""
    return _try_load()


def fallback_allowed() -> bool:
    return os.environ.get("HFREP_ALLOW_TORCH_FALLBACK", "0") == "1"


def native():
    """Return ``torch.ops.hfrep`` or raise loudly."""
    if not _try_load():
        raise RuntimeError(f"hfrep native kernel library unavailable: {_err!r}")
    return torch.ops.hfrep


def use_native_for(t: torch.Tensor) -> bool:
    """Decide the execution path for a tensor.

    CPU tensors -> reference path.  GPU tensors -> native path, raising if it cannot load
    (unless HFREP_ALLOW_TORCH_FALLBACK=1).
    """
    if t.device.type != "cuda":
        return False
    if _try_load():
        return True
    if fallback_allowed():
        return False
    raise RuntimeError(
        f"GPU tensor but hfrep native library failed to load ({_err!r}); refusing silent fallback. "
        "Build with `python build_native.py` or set HFREP_ALLOW_TORCH_FALLBACK=1 for debugging."
    )
