"""Training-run driver: logging, checkpoint/resume, NaN guard, fault injection, hipGraph replay.

The reference's loop (GAN/MTSS_WGAN_GP.py:254-287) trains for a fixed number of iterations,
prints every iteration and saves the generator once at the very end - a crash loses the run
(SURVEY.md §5).  :func:`run` wraps :class:`GANTrainer` with:

* structured JSONL logging every ``log_every`` iterations through deferred (non-blocking)
  device->host snapshots (:mod:`hfrep.utils.logger`);
* a NaN/Inf guard: a device-side finiteness flag of the losses, all-reduced across ranks together
  with the logged losses (averaged over ranks), so every rank stops at the same iteration (no rank
  is left waiting in a collective) and every rank logs the global-batch losses;
* periodic atomic checkpoints of the full training state (G, C, optimizer slots, the shared
  iteration counter, the RNG counter) by rank 0, keeping the newest ``keep`` files, and
  ``resume="auto"`` to continue from the newest one bitwise-identically;
* a fault-injection hook (``fault_at`` / ``HFREP_FAULT_AT=iteration[:rank]``) that raises
  :class:`InjectedFault` after a given iteration - used by the resume tests;
* optional hipGraph capture of the whole iteration (:class:`GraphedStep`): n_critic critic
  steps + the generator step replay as ONE graph launch, which removes the per-kernel launch
  cost that dominates at the reference batch of 32.
"""
from __future__ import annotations

import glob
import os
import time
from dataclasses import dataclass

import torch

from ..utils.checkpoint import apply_training_state, load_training_state, read_training_state, save_training_state
from ..utils.logger import AsyncScalars, JSONLLogger


class NonFiniteLoss(RuntimeError):
    pass


class InjectedFault(RuntimeError):
    pass


@dataclass
class RunOptions:
    epochs: int
    log_every: int = 100
    log_path: str | None = None
    echo: bool = True
    ckpt_dir: str | None = None
    ckpt_every: int = 0
    keep: int = 2
    resume: str | None = None          # path, or "auto" = newest checkpoint in ckpt_dir
    nan_guard: bool = True
    fault_at: int | None = None
    fault_rank: int = 0
    graph: bool = False


def _env_fault(opts: RunOptions):
    spec = os.environ.get("HFREP_FAULT_AT")
    if spec and opts.fault_at is None:
        it, _, rk = spec.partition(":")
        opts.fault_at, opts.fault_rank = int(it), int(rk or 0)


def latest_checkpoint(ckpt_dir: str) -> str | None:
    files = sorted(glob.glob(os.path.join(ckpt_dir, "state_*.pt")))
    return files[-1] if files else None


class GraphedStep:
    """Replays ``trainer.train_step`` from a captured hipGraph.

    Everything the step touches is device-resident and graph-safe: the Philox counter advances on
    the device, the optimizer's shared iteration counter is a device tensor, and every kernel runs
    on the current stream.  Only the host-side iteration count is bumped here.  The first
    ``warmup`` calls run the step eagerly (allocator and one-time kernel attributes settle), the
    next call captures it and from then on every call is one graph launch.
    """

    def __init__(self, trainer, warmup: int = 2):
        if trainer.device.type != "cuda":
            raise RuntimeError("graph capture needs a GPU trainer")
        if not trainer.rng.native:
            raise RuntimeError("graph capture needs the native (device-counter) RNG")
        if trainer.grad_sync is not None and trainer.world > 1:
            # RCCL collectives are graph-capturable (ProcessGroupNCCL records them on the captured
            # stream; tests/test_gpu_rccl.py replays them bitwise against the eager step on a 1-rank
            # communicator); gloo / CPU collectives are not.  Captured collectives across >= 2 real
            # GPUs have not been checked against the eager step yet (RCCL refuses two ranks on one
            # GPU, and the pool's boxes have one), so under DP the capture is opt-in:
            # HFREP_GRAPH_DP=1.  Without it a DP run replays nothing and steps eagerly.
            if not trainer.grad_sync.graph_capturable():
                raise RuntimeError("graph capture under data parallelism needs RCCL or the P2P all-reduce")
            if os.environ.get("HFREP_GRAPH_DP", "0") != "1":
                raise RuntimeError("graph capture under data parallelism is opt-in (HFREP_GRAPH_DP=1): multi-rank "
                                   "replay parity is unpinned")
        self.t, self.warmup, self.calls = trainer, warmup, 0
        self.graph = None

    def _capture(self):
        """Capture one step.

        The capture runs in THREAD-LOCAL mode: ProcessGroupNCCL's watchdog thread keeps polling
        the events of the warmup steps' collectives (``WorkNCCL::isCompleted`` ->
        ``hipEventQuery``), and in the default global mode any such query from another thread
        while a stream captures is illegal -- the watchdog then takes the process down (the
        round-2 driver run of tests/test_gpu_rccl.py).  Thread-local mode only forbids unsafe
        calls on the capturing thread.  Every outstanding bucket is joined, the device drained and every
        warmup collective confirmed complete (:meth:`GradSync.drain_`), and the captured bucket
        all-reduces go through a communicator that never runs eager work
        (:meth:`GradSync.use_graph_group_`): the watchdog has no event of a capturing stream to query."""
        t = self.t
        if t.grad_sync is not None:
            t.grad_sync.finish_()
        torch.cuda.synchronize()
        if t.grad_sync is not None:
            if not t.grad_sync.graph_capturable():  # a warmup bucket took gloo (P2P cap / dtype fallback)
                raise RuntimeError(f"graph capture: a gradient bucket went through {sorted(t.grad_sync.routes)}; "
                                   "gloo collectives cannot be captured (raise HFREP_DP_P2P_CAP or use RCCL)")
            t.grad_sync.drain_()
            t.grad_sync.use_graph_group_()
            torch.cuda.synchronize()
        it = t.iteration
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            t.train_step()
        if t.grad_sync is not None:
            t.grad_sync.forget_()
        t.iteration = it  # capture recorded the step, it did not run it

    def __call__(self):
        self.calls += 1
        if self.calls <= self.warmup:
            self.t.train_step()
            return
        if self.graph is None:
            self._capture()
        self.graph.replay()
        self.t.iteration += 1


def _log_tensors(trainer, nan_guard: bool) -> dict:
    """The logged loss scalars, averaged over ranks, and the all-ranks finiteness flag.

    One packed SUM all-reduce per log interval: [d_loss, d_real, d_fake, gp, g_loss..., finite]; a
    rank's non-finite loss makes the summed flag < world on every rank, so all ranks stop at the
    same iteration (no rank left waiting in a collective)."""
    d, g = trainer._d_acc.reshape(-1), trainer._g_acc.reshape(-1)
    if trainer.grad_sync is None or trainer.world <= 1:
        out = {"d": d, "g": g}
        if nan_guard:
            out["ok"] = (torch.isfinite(d).all() & torch.isfinite(g).all()).to(torch.float32).reshape(1)
        return out
    import torch.distributed as dist

    ok = (torch.isfinite(d).all() & torch.isfinite(g).all()).to(d.dtype).reshape(1)
    if nan_guard:
        # the run stops at this record anyway: a non-finite rank contributes zeros to the logged
        # mean and its flag (summed below) reports it
        pack = torch.cat([torch.nan_to_num(d, nan=0.0, posinf=0.0, neginf=0.0),
                          torch.nan_to_num(g.to(d.dtype), nan=0.0, posinf=0.0, neginf=0.0), ok])
    else:
        # unguarded runs log the raw mean, so a diverged rank shows up as NaN / Inf in the record
        pack = torch.cat([d, g.to(d.dtype), ok])
    dist.all_reduce(pack, op=dist.ReduceOp.SUM, group=trainer.grad_sync.group)
    nd, ng, w = d.numel(), g.numel(), float(trainer.world)
    out = {"d": pack[:nd] / w, "g": pack[nd:nd + ng] / w}
    if nan_guard:
        out["ok"] = (pack[nd + ng:] >= w - 0.5).to(torch.float32)
    return out


def resolve_resume(opts: RunOptions, trainer) -> str | None:
    """Checkpoint path to resume from.  Under data parallelism rank 0 resolves it (it is the rank
    that writes checkpoints) and broadcasts the path, so every rank resumes the same iteration even
    while rank 0 rotates files."""
    if not opts.resume:
        return None
    if opts.resume == "auto" and not opts.ckpt_dir:
        raise ValueError("resume='auto' needs ckpt_dir")
    path = None
    if trainer.rank == 0 or trainer.grad_sync is None:
        path = latest_checkpoint(opts.ckpt_dir) if opts.resume == "auto" else opts.resume
    if trainer.grad_sync is not None and trainer.world > 1:
        import torch.distributed as dist

        box = [path]
        dist.broadcast_object_list(box, src=0, group=trainer.grad_sync.group)
        path = box[0]
    return path


def resume_state(path: str, trainer) -> None:
    """Load the training state at ``path`` on every rank.

    With a shared checkpoint directory each rank reads the file itself.  When some rank cannot see
    it (``ckpt_dir`` is local to rank 0's node or filesystem), rank 0 reads it and broadcasts the
    state, so a rank-local ``ckpt_dir`` works too."""
    if trainer.grad_sync is None or trainer.world <= 1:
        load_training_state(path, trainer)
        return
    import torch.distributed as dist

    seen = torch.tensor([1.0 if os.path.exists(path) else 0.0], dtype=torch.float64)
    if trainer.grad_sync.backend == "nccl":
        seen = seen.to(trainer.device)
    dist.all_reduce(seen, op=dist.ReduceOp.MIN, group=trainer.grad_sync.group)
    if float(seen.item()) > 0.5:
        load_training_state(path, trainer)
        return
    box = [read_training_state(path) if trainer.rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=trainer.grad_sync.group)
    apply_training_state(box[0], trainer)


def run(trainer, opts: RunOptions, logger: JSONLLogger | None = None) -> list[dict]:
    """Train until ``trainer.iteration == opts.epochs``; returns the emitted log records."""
    _env_fault(opts)
    own_logger = logger is None
    logger = logger or JSONLLogger(opts.log_path, rank=trainer.rank, echo=opts.echo)
    records: list[dict] = []

    gs = trainer.grad_sync

    def emit(rec):
        if rec is None:
            return
        if "ok" in rec:
            ok = rec.pop("ok")
            if opts.nan_guard and not ok:
                logger.log({"event": "nonfinite_loss", "iteration": rec["iteration"]})
                if gs is not None:
                    # a failed P2P all-reduce writes NaN gradients: name the cause when it is that
                    gs.check_errors(blocking=True)
                raise NonFiniteLoss(f"non-finite loss by iteration {rec['iteration']}")
        d = rec.pop("d", None)
        g = rec.pop("g", None)
        if d is not None:
            rec.update(d_loss=d[0], d_real=d[1], d_fake=d[2], gp=d[3], g_loss=g if not isinstance(g, list) else g[0])
        records.append(rec)
        logger.log(rec)

    path = resolve_resume(opts, trainer)
    if path:
        resume_state(path, trainer)
        logger.log({"event": "resumed", "path": path, "iteration": trainer.iteration})
    step = GraphedStep(trainer) if opts.graph else trainer.train_step
    snap = AsyncScalars()
    wpi = trainer.windows_per_iteration() * trainer.world
    t_last, it_last = time.time(), trainer.iteration
    try:
        while trainer.iteration < opts.epochs:
            step()
            it = trainer.iteration
            if opts.fault_at is not None and it == opts.fault_at and trainer.rank == opts.fault_rank:
                logger.log({"event": "injected_fault", "iteration": it})
                raise InjectedFault(f"injected fault after iteration {it} on rank {trainer.rank}")
            if it % opts.log_every == 0 or it == opts.epochs:
                now = time.time()
                meta = {"iteration": it, "windows_per_s": wpi * (it - it_last) / max(now - t_last, 1e-9)}
                t_last, it_last = now, it
                if gs is not None:
                    gs.check_errors()  # non-blocking: raises P2PTimeout once a give-up has reached the host
                emit(snap.snapshot(meta, **_log_tensors(trainer, opts.nan_guard)))
            if opts.ckpt_dir and opts.ckpt_every and it % opts.ckpt_every == 0:
                states = _gather_host_rng(trainer)
                if trainer.rank == 0:
                    _checkpoint(trainer, opts, states)
                if trainer.grad_sync is not None and trainer.world > 1:
                    import torch.distributed as dist

                    dist.barrier(group=trainer.grad_sync.group)  # the file exists before any rank goes on
        emit(snap.collect())
        if gs is not None:
            gs.check_errors(blocking=True)
    finally:
        if own_logger:
            logger.close()
    return records


def checkpoint_now(trainer, opts: RunOptions) -> str | None:
    """Checkpoint the current iteration into ``opts.ckpt_dir`` (all ranks call; rank 0 writes), unless
    the periodic checkpoint of this iteration already exists."""
    if not opts.ckpt_dir:
        return None
    path = os.path.join(opts.ckpt_dir, f"state_{trainer.iteration:09d}.pt")
    states = _gather_host_rng(trainer)
    if trainer.rank == 0 and not os.path.exists(path):
        path = _checkpoint(trainer, opts, states)
    if trainer.grad_sync is not None and trainer.world > 1:
        import torch.distributed as dist

        dist.barrier(group=trainer.grad_sync.group)
    return path


def _gather_host_rng(trainer):
    """Every rank's host-RNG state (None with the device counter RNG or a single process)."""
    if trainer.rng.native or trainer.grad_sync is None or trainer.world <= 1:
        return None
    import torch.distributed as dist

    states = [None] * trainer.world
    dist.all_gather_object(states, trainer.rng.gen.get_state(), group=trainer.grad_sync.group)
    return states


def _checkpoint(trainer, opts: RunOptions, rng_states=None) -> str:
    os.makedirs(opts.ckpt_dir, exist_ok=True)
    path = os.path.join(opts.ckpt_dir, f"state_{trainer.iteration:09d}.pt")
    save_training_state(path, trainer, rng_states)
    old = sorted(glob.glob(os.path.join(opts.ckpt_dir, "state_*.pt")))[:-opts.keep]
    for p in old:
        os.remove(p)
    return path
