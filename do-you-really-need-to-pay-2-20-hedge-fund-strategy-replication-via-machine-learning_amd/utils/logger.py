"""Structured run logging (SURVEY.md §5 "Metrics / logging / observability").

The reference prints ``"%d [D loss: %f] [G loss: %f]"`` every iteration (GAN/MTSS_WGAN_GP.py:284),
which on a GPU means one blocking device->host copy per step.  Here:

* :class:`AsyncScalars` snapshots device scalars into pinned host memory with a non-blocking copy
  and an event; the values are read one log interval later, when the copy has long completed, so
  logging never stalls the stream;
* :class:`JSONLLogger` appends one JSON object per record (rank 0 only by default) and can echo
  the reference's console line.
"""
from __future__ import annotations

import json
import os
import time

import torch


class AsyncScalars:
    """Deferred device->host snapshot of a few scalar tensors."""

    def __init__(self):
        self._pending = None  # (meta, host tensors, event)

    def snapshot(self, meta: dict, **tensors) -> dict | None:
        """Queue a copy of ``tensors``; returns the PREVIOUS snapshot's values (or None)."""
        prev = self.collect()
        host, ev = {}, None
        for k, t in tensors.items():
            t = t.detach().reshape(-1).float()
            if t.is_cuda:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                h.copy_(t, non_blocking=True)
            else:
                h = t.clone()
            host[k] = h
        if any(t.is_cuda for t in tensors.values()):
            ev = torch.cuda.Event()
            ev.record()
        self._pending = (dict(meta), host, ev)
        return prev

    def collect(self) -> dict | None:
        """Values of the pending snapshot (waits for its copy if still in flight)."""
        if self._pending is None:
            return None
        meta, host, ev = self._pending
        self._pending = None
        if ev is not None:
            ev.synchronize()
        out = dict(meta)
        for k, h in host.items():
            v = h.tolist()
            out[k] = v[0] if len(v) == 1 else v
        return out


class JSONLLogger:
    """Append-only JSON-lines log.  ``echo`` prints the reference-style console line as well."""

    def __init__(self, path: str | None, rank: int = 0, echo: bool = True, all_ranks: bool = False):
        self.rank = rank
        self.active = all_ranks or rank == 0
        self.echo = echo and self.active
        self.path = path
        self._fh = None
        if path and self.active:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def log(self, rec: dict) -> None:
        if not self.active:
            return
        rec = dict(rec)
        rec.setdefault("time", time.time())
        if self.rank:
            rec.setdefault("rank", self.rank)
        if self._fh is not None:
            self._fh.write(json.dumps(rec, default=float) + "\n")
        if self.echo and "iteration" in rec and "d_loss" in rec:
            print("%d [D loss: %f] [G loss: %f]" % (rec["iteration"] - 1, rec["d_loss"], rec["g_loss"]), flush=True)
        elif self.echo and "event" in rec:
            print(f"[hfrep] {rec['event']}: " + ", ".join(f"{k}={v}" for k, v in rec.items()
                                                          if k not in ("event", "time")), flush=True)

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_jsonl(path: str) -> list[dict]:
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]
