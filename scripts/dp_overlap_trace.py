"""Bench-shape data-parallel step with the RCCL gradient sync, for a rocprofv3 kernel timeline.

One GPU cannot host two RCCL ranks, so a 1-rank ``nccl`` process group stands in (as in
tests/test_gpu_rccl.py): ``GradSync`` is told the job has 2 ranks, which sends both gradient buckets of
every model update through ``all_reduce(AVG)`` on RCCL's own stream, launched from the reverse pass
(train/gan_trainer.py ``_hook``).  Run it under ``rocprofv3 --kernel-trace`` and summarise the trace with
``scripts/dp_overlap_summary.py``: every RCCL kernel is listed with the compute kernels it overlapped
in time on the other queue.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python scripts/dp_overlap_trace.py
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--steps", type=int, default=1, help="traced steps after the warmup")
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import hfrep  # noqa: F401
    from hfrep.data.windows import synthetic_windows
    from hfrep.parallel.dp import GradSync, nccl_graph_safe_env
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(s.getsockname()[1])
    s.close()
    nccl_graph_safe_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ds = synthetic_windows(8192, 24, 32, seed=1234)
    cfg = GANConfig(arch="lstm", loss="wgan_gp", window=24, features=32, batch_size=a.batch, dtype=a.dtype, seed=123)
    tr = GANTrainer(cfg, ds, device=dev)
    tr.grad_sync = GradSync(dist.group.WORLD, 2, buckets=2)
    for _ in range(a.warmup):
        tr.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    rec = tr.losses()
    print(f"[dp_overlap_trace] B={a.batch} {a.dtype}: {ms:.1f} ms / step with the 2-bucket RCCL sync; "
          f"losses finite: {all(np.isfinite(v) for v in rec.values())}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
