"""Latency of the one-shot IPC all-reduce (csrc/p2p.hip) with W processes sharing one GPU.

    python scripts/bench_p2p.py --world 8 [--floats 140000,1048576] [--iters 200]

Every rank binds cuda:0 (the gpurun boxes have one MI355X; RCCL refuses shared-GPU ranks), so this
prices the kernel's staging, flag hand-off and W-way summation -- not xGMI bandwidth.  Each size is
timed as a hipGraph of ``iters`` back-to-back calls (after a warmup), rank 0 prints one JSON line.
"""
import argparse
import json
import os
import socket
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def worker(rank, world, port, sizes, iters, q):
    import torch
    import torch.distributed as dist

    import hfrep  # noqa: F401
    from hfrep.parallel.p2p import P2PAllReduce

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ar = P2PAllReduce(dist.group.WORLD, cap=max(sizes), device=dev)
    out = []
    for n in sizes:
        x = torch.randn(n, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                ar.all_reduce_(x, average=True)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                ar.all_reduce_(x, average=True)
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        t = torch.tensor([us])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out.append({"world": world, "floats": n, "bytes": 4 * n, "us_per_call_max_rank": round(float(t), 2)})
    ar.check()
    dist.barrier()
    ar.close()
    dist.destroy_process_group()
    if rank == 0:
        q.put(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--floats", default="140000,1048576")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    sizes = [int(v) for v in a.floats.split(",")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, sizes, a.iters, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
    for r in res:
        print(json.dumps(r), flush=True)
    return 0 if all(p.exitcode == 0 for p in ps) else 1


if __name__ == "__main__":
    sys.exit(main())
