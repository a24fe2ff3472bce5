"""Result collection for the spawn-based multi-process tests.

A child that dies (abort, segfault, an RCCL watchdog ``terminate``) never puts its result on the
queue; waiting on ``q.get(timeout=...)`` alone then burns the whole timeout and reports
``_queue.Empty`` instead of the child's exit code.  :func:`gather` polls the queue in short slices
and checks the children between slices, so a dead child fails the test within seconds and names
its exit code.
"""
from __future__ import annotations

import queue
import time


def gather(procs, q, n: int, timeout: float = 300.0, poll: float = 1.0) -> list:
    """``n`` results from ``q``; raises as soon as a child has exited non-zero (or every child has
    exited) without the results being complete, or when ``timeout`` seconds pass."""
    out: list = []
    deadline = time.monotonic() + timeout
    try:
        while len(out) < n:
            try:
                out.append(q.get(timeout=poll))
                continue
            except queue.Empty:
                pass
            dead = [p for p in procs if p.exitcode is not None and p.exitcode != 0]
            if dead or all(p.exitcode is not None for p in procs):
                # a result put just before the exit may still be in the pipe: one last short drain
                try:
                    while len(out) < n:
                        out.append(q.get(timeout=poll))
                except queue.Empty:
                    pass
                if len(out) < n:
                    codes = {p.pid: p.exitcode for p in procs}
                    raise AssertionError(f"child process(es) exited without a result: exit codes {codes}; "
                                         f"got {len(out)} of {n} results")
            if time.monotonic() > deadline:
                raise AssertionError(f"timed out after {timeout:.0f} s with {len(out)} of {n} results")
        return out
    finally:
        for p in procs:
            p.join(timeout=30 if len(out) == n else 1)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
