"""Data-parallel training over RCCL (xGMI) — one process per GPU.

The reference has no parallelism at all.  Here every rank runs the full GAN
step on its own per-GPU batch (rank-seeded Philox streams), and each model's gradients — ONE
flat fp32 buffer per model, ~0.55 MB for the LSTM critic — are averaged before the fused
optimizer launch.  At this message size the ring is latency-bound, so the buffer
is cut into just two buckets at layer boundaries (``Sequential.grad_buckets``): each is
all-reduced asynchronously from the reverse pass as soon as its layers are final (the reduction
of the last layers overlaps the backward of the first ones), and :meth:`GradSync.finish_` joins
them before the optimizer.  No per-parameter collectives.

``torch.distributed`` with backend ``nccl`` is RCCL on ROCm; ``gloo`` is used for CPU tests.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world) from torchrun-style environment variables."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def nccl_graph_safe_env() -> None:
    """Environment for RCCL collectives inside hipGraph captures; set before the process group exists.

    ProcessGroupNCCL recycles its completion events through a cache.  A collective captured into a
    graph can then RE-RECORD (inside the capture) the event of an eager warmup collective that the
    watchdog thread still holds; the watchdog's next ``hipEventQuery`` on it fails with
    hipErrorCapturedEvent ("operation not permitted on an event last recorded in a capturing
    stream") and the watchdog terminates the process -- tests/test_gpu_rccl.py::
    test_rccl_grad_sync_in_graph failed this way once in six round-3 runs.  Without the cache every
    work owns its events, and captured collectives are never enqueued to the watchdog."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init_distributed(backend: str | None = None, timeout_s: float = 600.0):
    """Initialise the default process group from the environment (env://).

    Returns (rank, local_rank, world, group).  With WORLD_SIZE == 1 nothing is initialised.
    """
    rank, local_rank, world = env_rank()
    if world <= 1:
        return rank, local_rank, world, None
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # torchrun always sets MASTER_PORT; a hand-launched job names it with HFREP_MASTER_PORT (no
    # fixed default: two jobs on one node would silently rendezvous with each other)
    if "MASTER_PORT" not in os.environ:
        if "HFREP_MASTER_PORT" not in os.environ:
            raise RuntimeError("WORLD_SIZE > 1 needs MASTER_PORT (torchrun sets it) or HFREP_MASTER_PORT")
        os.environ["MASTER_PORT"] = os.environ["HFREP_MASTER_PORT"]
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        # surface RCCL errors as Python exceptions instead of hanging a collective forever
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        nccl_graph_safe_env()
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(**kw)
    return rank, local_rank, world, dist.group.WORLD


class GradSync:
    """Averages flat gradient buckets across ranks (one collective per model per step)."""

    def __init__(self, group, world: int, buckets: int = 2):
        self.group, self.world, self.buckets = group, world, buckets
        self.backend = dist.get_backend(group) if group is not None else None
        # the group the gradient buckets go through: ``group``, or after :meth:`use_graph_group_` a
        # second communicator over the same ranks that only ever runs inside hipGraph captures
        self.bucket_group = group
        self._graph_group = None
        self._pending = []
        # the newest async work: RCCL runs a group's collectives on one stream in issue order, so its
        # completion implies every earlier one's (graph capture waits for it, drain_)
        self._last = None
        # HFREP_DP_P2P=1: buckets of <= HFREP_DP_P2P_CAP floats go through the one-shot IPC all-reduce
        # (parallel/p2p.py, csrc/p2p.hip) on a side stream instead of RCCL; built at the first bucket
        # (HFREP_DP_P2P=force: any process group carries the handles -- gloo ranks sharing one GPU in
        # scripts/bench_dp_shared.py; the buckets must be CUDA tensors of processes on one node)
        mode = os.environ.get("HFREP_DP_P2P", "0")
        self.use_p2p = world > 1 and ((mode == "1" and self.backend == "nccl") or mode == "force")
        self.p2p_cap = int(os.environ.get("HFREP_DP_P2P_CAP", str(1 << 21)))
        self.p2p = None
        self._p2p_stream = None
        # the collective kinds the buckets actually took ("p2p", "rccl", "gloo"): a bucket over the P2P cap,
        # or not a CUDA fp32 tensor, falls back to the group's collective even with HFREP_DP_P2P on, which
        # decides what a hipGraph capture may contain (use_graph_group_, graph_capturable)
        self.routes: set = set()
        # exposed-wait timing (bench.py): per finish_ an event pair on the compute stream around the join
        self.timing = False
        self._events = []

    def _p2p_for(self, t: torch.Tensor):
        """The one-shot all-reduce for bucket ``t`` (None: RCCL).  The first call is collective."""
        if not self.use_p2p or t.numel() > self.p2p_cap or not t.is_cuda or t.dtype != torch.float32:
            return None
        if self.p2p is None:
            from .p2p import P2PAllReduce

            self.p2p = P2PAllReduce(self.group, cap=self.p2p_cap, device=t.device)
            self._p2p_stream = torch.cuda.Stream(device=t.device)
        return self.p2p

    def all_reduce_(self, flat_grad: torch.Tensor) -> None:
        if self.world <= 1:
            return
        p2p = self._p2p_for(flat_grad)
        self.routes.add("p2p" if p2p is not None else "rccl" if self.backend == "nccl" else "gloo")
        if p2p is not None:
            p2p.all_reduce_(flat_grad, average=True)
        elif self.backend == "nccl":
            dist.all_reduce(flat_grad, op=dist.ReduceOp.AVG, group=self.bucket_group)
        else:
            dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)
            flat_grad.div_(self.world)

    # ---- bucketed, overlapped reduction -------------------------------------------------------
    def start_(self, grad_slice: torch.Tensor):
        """Launch the average of one gradient bucket without blocking the compute stream.

        ProcessGroupNCCL orders the collective after the work already queued on the current
        stream and runs it on its own stream, so the backward of the remaining (earlier) layers
        keeps running while this bucket is reduced over xGMI; :meth:`finish_` makes the compute
        stream wait for all launched buckets before the optimizer reads the gradients.
        """
        if self.world <= 1:
            return
        p2p = self._p2p_for(grad_slice)
        self.routes.add("p2p" if p2p is not None else "rccl" if self.backend == "nccl" else "gloo")
        if p2p is not None:
            # the side stream joins the compute stream here and is joined back in finish_
            s = self._p2p_stream
            s.wait_stream(torch.cuda.current_stream(grad_slice.device))
            with torch.cuda.stream(s):
                p2p.all_reduce_(grad_slice, average=True)
            self._pending.append(("p2p", s))
        elif self.backend == "nccl":
            w = dist.all_reduce(grad_slice, op=dist.ReduceOp.AVG, group=self.bucket_group, async_op=True)
            self._pending.append(w)
            self._last = w
        else:
            self._pending.append((dist.all_reduce(grad_slice, op=dist.ReduceOp.SUM, group=self.group,
                                                  async_op=True), grad_slice))

    def finish_(self) -> int:
        n = len(self._pending)
        timed = self.timing and n > 0 and self._pending_on_gpu()
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        for w in self._pending:
            if isinstance(w, tuple) and w[0] == "p2p":
                torch.cuda.current_stream(w[1].device).wait_stream(w[1])
            elif isinstance(w, tuple):
                w[0].wait()
                w[1].div_(self.world)
            else:
                w.wait()
        self._pending = []
        if timed:
            e1.record()
            self._events.append((e0, e1))
        return n

    def _pending_on_gpu(self) -> bool:
        return torch.cuda.is_available() and (self.backend == "nccl" or self.p2p is not None)

    def exposed_wait_ms(self, reset: bool = True) -> float:
        """Total time the compute stream spent waiting for bucket all-reduces at :meth:`finish_` since the
        last reset (the non-overlapped part of the gradient averaging; needs ``timing = True``).
        Synchronises on the recorded events."""
        tot = 0.0
        for e0, e1 in self._events:
            e1.synchronize()
            tot += e0.elapsed_time(e1)
        if reset:
            self._events = []
        return tot

    def graph_capturable(self) -> bool:
        """Whether a step's bucket all-reduces can be captured into a hipGraph at all: RCCL collectives, or
        every bucket on the one-shot P2P kernel (device-side epochs; the group only carried the IPC
        handles).  gloo collectives cannot be captured -- also not a bucket that fell back to gloo from
        the P2P route during the eager steps (``routes``)."""
        if self.world <= 1:
            return True
        if "gloo" in self.routes:
            return False
        return self.backend == "nccl" or self.use_p2p

    def check_errors(self, blocking: bool = False) -> None:
        """Surface a failed one-shot all-reduce (P2PTimeout).  Non-blocking by default (pinned-host
        snapshot of the error word, see P2PAllReduce.poll); the runner calls it at every log record."""
        if self.p2p is None:
            return
        if blocking:
            self.p2p.check()
        else:
            self.p2p.poll()

    def close(self) -> None:
        """Collective teardown of the P2P communicator (every rank, same point); RCCL groups are left
        to ``destroy_process_group``."""
        if self.p2p is not None:
            self.p2p.close()
            self.p2p = None

    def drain_(self, timeout_s: float = 120.0) -> bool:
        """Block the host until the newest async collective (hence every earlier one of the group) has
        COMPLETED on the device (``Work.is_completed``: its end event has been reached), so no eager
        collective is in flight when a hipGraph capture starts.  Deterministic -- no timing assumption
        about the ProcessGroupNCCL watchdog thread: with its event cache off (:func:`nccl_graph_safe_env`)
        an event the watchdog still queries is never re-recorded inside the capture.  Call it outside
        any capture; raises if the work does not complete within ``timeout_s``."""
        import time

        w, self._last = self._last, None
        if w is None:
            return False
        t0 = time.monotonic()
        while not w.is_completed():
            if time.monotonic() - t0 > timeout_s:
                raise RuntimeError(f"GradSync.drain_: a collective did not complete within {timeout_s} s")
            time.sleep(0.0005)
        return True

    def needs_graph_group(self) -> bool:
        """Whether a capture needs the capture-only communicator (:meth:`use_graph_group_`): any RCCL
        bucket would be captured.  Not when every bucket of the eager steps went through the P2P kernel
        (no RCCL work inside the capture); a bucket over HFREP_DP_P2P_CAP (or not CUDA fp32) went to
        RCCL instead and would be captured on the eager communicator, so it does."""
        if self.backend != "nccl" or self.world <= 1 or self.group is None:
            return False
        return not (self.use_p2p and self.routes and self.routes <= {"p2p"})

    def use_graph_group_(self) -> bool:
        """Route the bucket all-reduces through a communicator reserved for hipGraph captures.

        ProcessGroupNCCL's watchdog thread keeps querying the end events of a group's eager collectives
        until it retires them, and HIP refuses ``hipEventQuery`` on an event of a stream that is being
        captured (hipErrorCapturedEvent, which the watchdog turns into an abort) -- the captured
        collectives pull the group's RCCL stream into the capture.  Whether the watchdog has retired
        the warmup works before the capture starts is timing (round 3 slept 0.3 s; round 4's
        completion poll alone failed on the GPU).  A second group over the same ranks, connected
        eagerly and used ONLY inside captures, has no eager work for its watchdog to query, and the
        first group's stream never joins a capture: no timing assumption left.  Collective call (every
        rank, same point); nccl only.  Returns whether the switch happened."""
        if not self.needs_graph_group():
            return False
        if self._graph_group is None:
            ranks = dist.get_process_group_ranks(self.group)
            dev = torch.device("cuda", torch.cuda.current_device())
            self._graph_group = dist.new_group(ranks=ranks, backend="nccl", device_id=dev)
        self.bucket_group = self._graph_group
        return True

    def forget_(self) -> None:
        """Drop the newest-work reference (after a capture: captured works must never be queried)."""
        self._last = None

    def broadcast_params(self, models, src: int = 0) -> None:
        if self.world <= 1:
            return
        for m in models:
            with torch.no_grad():
                dist.broadcast(m.flat.data, src=src, group=self.group)

    def all_reduce_scalar(self, x: float, op=dist.ReduceOp.MAX, device=None) -> float:
        if self.world <= 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=op, group=self.group)
        return float(t.item())
