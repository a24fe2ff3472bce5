"""One-shot peer-to-peer all-reduce for small gradient buckets (the optional custom
xGMI collective beside RCCL).

The reference trains on one device (``GAN/MTSS_WGAN_GP.py:254-287`` has no collective at all); the
data-parallel framework averages one ~0.5 MB flat gradient bucket per model per step.  At that size a
ring all-reduce is latency-bound (2 (W - 1) link hops), while on the MI355X node's fully connected
xGMI mesh each rank can read all peers' buckets at once.  ``csrc/p2p.hip`` implements that: every
rank exports one fine-grained device buffer through a HIP IPC handle, every peer maps it, and one
kernel per call stages the local bucket, raises one flag per (peer, block), waits for the peers'
flags (bounded: a missing peer sets an error word instead of hanging) and sums the W staged buckets
in rank order -- every rank gets the same bits.  The epoch counter lives in device memory, so the
call can be captured into a hipGraph.

The handles are exchanged once over any process group (gloo in the tests, the RCCL group in
training).  Used by :class:`hfrep.parallel.dp.GradSync` when ``HFREP_DP_P2P=1`` (RCCL otherwise).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _native

MAX_RANKS = 8


class P2PAllReduce:
    """Sum / average fp32 tensors of up to ``cap`` elements across the ranks of ``group``.

    Collective to construct (every rank, same ``cap``); every rank must then issue the same sequence of
    :meth:`all_reduce_` calls with the same sizes.  All ranks must be on one node (IPC)."""

    def __init__(self, group=None, cap: int = 1 << 20, device: torch.device | None = None):
        self.group = group
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

    def all_reduce_(self, x: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In place: x = sum (or mean) over ranks.  Launches one kernel on the current stream."""
        if x.numel() > self.cap:
            raise ValueError(f"P2PAllReduce: {x.numel()} elements exceed cap {self.cap}")
        self._ops.p2p_allreduce_(x, self.buf, self.peers, self.rank, self.cap, 1.0 / self.world if average else 1.0)
        return x

    def check(self) -> None:
        """Raise if any call since the last check gave up waiting for a peer (synchronises)."""
        if int(self._ops.p2p_error(self.buf)):
            raise RuntimeError("P2PAllReduce: a peer's flag did not arrive (peer missing or out of step)")

    def close(self) -> None:
        for p in self._opened:
            self._ops.p2p_close(p)
        self._opened = []
