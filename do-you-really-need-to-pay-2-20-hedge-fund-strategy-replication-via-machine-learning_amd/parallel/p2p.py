"""One-shot peer-to-peer all-reduce for small gradient buckets (the optional custom
xGMI collective beside RCCL).

The reference trains on one device (``GAN/MTSS_WGAN_GP.py:254-287`` has no collective at all); the
data-parallel framework averages one ~0.5 MB flat gradient bucket per model per step.  At that size a
ring all-reduce is latency-bound (2 (W - 1) link hops), while on the MI355X node's fully connected
xGMI mesh each rank can read all peers' buckets at once.  ``csrc/p2p.hip`` implements that: every
rank exports one fine-grained device buffer through a HIP IPC handle, every peer maps it, and one
kernel per call stages the local bucket, raises one flag per (peer, block), waits for the peers'
flags and sums the W staged buckets in rank order -- every rank gets the same bits.  The epoch
counter lives in device memory, so the call can be captured into a hipGraph.

Failure is loud: a wait is bounded by wall-clock time (``HFREP_P2P_TIMEOUT_S``, default 30 s); the
block that gives up poisons every rank's error word, every rank's waiting blocks leave at once,
every unfinished chunk of the output is written as NaN (so the runner's NaN guard stops all ranks at
the next log record, graph replays included), and every later call on the poisoned communicator
returns NaN without waiting.  :meth:`P2PAllReduce.poll` reads the error word through a pinned-host
copy without blocking the host and raises :class:`P2PTimeout`; :meth:`check` does the same
synchronously.  A poisoned communicator is not reused (close it and build a new one).

The handles are exchanged once over any process group (gloo in the tests, the RCCL group in
training).  Used by :class:`hfrep.parallel.dp.GradSync` when ``HFREP_DP_P2P=1`` (RCCL otherwise).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops import _native

MAX_RANKS = 8
ERR_OFFSET = 256  # csrc/kernels.h kP2PErr: byte offset of the error word in each rank's buffer


class P2PTimeout(RuntimeError):
    """A P2P all-reduce gave up waiting for a peer (peer missing, late past the timeout, or out of step)."""


def default_timeout_s() -> float:
    return float(os.environ.get("HFREP_P2P_TIMEOUT_S", "30"))


class P2PAllReduce:
    """Sum / average fp32 tensors of up to ``cap`` elements across the ranks of ``group``.

    Collective to construct (every rank, same ``cap``); every rank must then issue the same sequence of
    :meth:`all_reduce_` calls with the same sizes.  All ranks must be on one node (IPC)."""

    def __init__(self, group=None, cap: int = 1 << 20, device: torch.device | None = None,
                 timeout_s: float | None = None):
        self.group = group
        self.timeout_s = float(timeout_s if timeout_s is not None else default_timeout_s())
        if not self.timeout_s > 0:
            raise ValueError("P2PAllReduce: timeout_s must be positive")
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > MAX_RANKS:
            raise ValueError(f"P2PAllReduce: at most {MAX_RANKS} ranks (one node), got {self.world}")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device, self.cap = dev, int(cap)
        ops = _native.native()
        self._ops = ops
        self.buf = ops.p2p_buffer(self.cap, dev.index)
        own = self.buf.data_ptr()
        handles = [None] * self.world
        dist.all_gather_object(handles, list(ops.p2p_handle(self.buf)), group=group)
        self._opened = []
        peers = []
        for r, h in enumerate(handles):
            if r == self.rank:
                peers.append(own)
            else:
                p = int(ops.p2p_open(h, dev.index))
                self._opened.append(p)
                peers.append(p)
        self.peers = peers
        # asynchronous error-word snapshots (poll): device word -> pinned host int, ordered by an event
        self._err_dev = self.buf[ERR_OFFSET:ERR_OFFSET + 4].view(torch.int32)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_evt = None

    def all_reduce_(self, x: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In place: x = sum (or mean) over ranks.  Launches one kernel on the current stream."""
        if x.numel() > self.cap:
            raise ValueError(f"P2PAllReduce: {x.numel()} elements exceed cap {self.cap}")
        if self.buf is None:
            raise RuntimeError("P2PAllReduce: closed")
        self._ops.p2p_allreduce_(x, self.buf, self.peers, self.rank, self.cap, 1.0 / self.world if average else 1.0,
                                 self.timeout_s)
        return x

    def _raise(self, word: int) -> None:
        raise P2PTimeout(f"P2PAllReduce (rank {self.rank}): rank {word - 1} gave up waiting for a peer after "
                         f"{self.timeout_s:g} s (peer missing, late or out of step); the buffers were poisoned "
                         f"and the reduced tensors hold NaN")

    def check(self) -> None:
        """Raise :class:`P2PTimeout` if any call so far gave up (synchronous; the word is sticky)."""
        if self.buf is None:
            return
        w = int(self._ops.p2p_error(self.buf))
        if w:
            self._raise(w)

    def poll(self) -> None:
        """Non-blocking check: raise if an earlier snapshot of the error word has landed and is set, then
        take a new snapshot (device -> pinned host copy on the current stream, after the calls issued so
        far).  Call it at log intervals; a failure surfaces at most two intervals late."""
        if self.buf is None:
            return
        if self._err_evt is not None:
            if not self._err_evt.query():
                return  # the previous snapshot is still in flight
            w = int(self._err_host[0])
            self._err_evt = None
            if w:
                self._raise(w)
        self._err_host.copy_(self._err_dev, non_blocking=True)
        self._err_evt = torch.cuda.Event()
        self._err_evt.record()

    def close(self) -> None:
        """Collective teardown (every rank): finish this rank's kernels, wait until every rank has
        finished its own (peers write flags into our buffer and read our slots), unmap the peers'
        buffers, and wait again before the own buffer may be freed."""
        if self.buf is None:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        for p in self._opened:
            self._ops.p2p_close(p)
        self._opened = []
        dist.barrier(group=self.group)
        self._err_evt = None
        self._err_dev = None
        self.buf = None  # the tensor's deleter frees the allocation
