"""Two-process data-parallel training step with the gradient buckets on the one-shot IPC all-reduce
(csrc/p2p.hip), for a rocprofv3 kernel timeline: both ranks share the box's one GPU (gloo carries the
handle exchange and the scalars), each rank's buckets run on its side stream while its reverse pass
continues on the compute stream.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run_%pid% -- python scripts/dp_p2p_trace.py
    python scripts/dp_overlap_summary.py OUT/.../<pid>_kernel_trace.csv     (one file per rank)

The parent only spawns the ranks; it never touches the GPU.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def worker(rank, world, port, batch, dtype, warmup, steps, q):
    import traceback

    try:
        import time

        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.data.windows import synthetic_windows
        from hfrep.train.gan_trainer import GANConfig, GANTrainer

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ds = synthetic_windows(8192, 24, 32, seed=1234)
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=24, features=32, batch_size=batch, dtype=dtype, seed=123)
        tr = GANTrainer(cfg, ds, device=dev, process_group=dist.group.WORLD, rank=rank, world=world)
        tr.grad_sync.use_p2p = True
        for _ in range(warmup):
            tr.train_step()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.train_step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        tr.grad_sync.p2p.check()
        dist.barrier()
        tr.grad_sync.p2p.close()
        dist.destroy_process_group()
        q.put({"rank": rank, "ms_per_step": round(ms, 2), "pid": os.getpid()})
    except Exception:
        q.put(traceback.format_exc())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    import json

    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, a.batch, a.dtype, a.warmup, a.steps, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        print(json.dumps(r) if isinstance(r, dict) else r, flush=True)
    return 0 if all(isinstance(r, dict) for r in res) and all(p.exitcode == 0 for p in ps) else 1


if __name__ == "__main__":
    sys.exit(main())
