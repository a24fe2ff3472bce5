"""Data-parallel overhead at equal total work, on ONE GPU: 2 ranks x B/2 windows vs 1 rank x B.

RCCL refuses two ranks on one GPU, so the ranks share cuda:0 over a gloo group and average their
gradient buckets with the one-shot P2P all-reduce (HFREP_DP_P2P=force, csrc/p2p.hip).  Each rank runs
bench.py's timed loop (`bench._measure`: warmup, barrier + sync on both sides, MAX over ranks); the
single-rank run at the full batch is the reference.  The two ranks' kernels share the device, so the
2-rank time is the sum of both halves' work plus the DP overhead (bucket kernels, stream joins, the
rank skew at each all-reduce), and `allreduce_exposed_ms_per_step` is each rank's compute-stream wait.

usage: python scripts/bench_dp_shared.py [--batch 262144] [--steps 5] [--warmup 2] [--dtype float32]
"""
import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _args(a, batch):
    return argparse.Namespace(window=24, features=32, batch_per_gpu=batch, hidden=100, model="mtss_wgan_gp",
                              dataset_windows=8192, warmup=a.warmup, steps=a.steps, trace_out="", profile_steps=0)


def _worker(rank, world, port, a, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0", HFREP_DP_P2P="force")
        import torch
        import torch.distributed as dist

        import bench
        import hfrep  # noqa: F401

        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        out = bench._measure(_args(a, a.batch // world), a.dtype, rank, world, dist.group.WORLD,
                             torch.device("cuda", 0))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--world", type=int, default=2)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _spawn import gather

    # 1 rank x B (a child process too: the two runs never share an allocator)
    ctx = mp.get_context("spawn")
    for world in (1, a.world):
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        q = ctx.Queue()
        procs = [ctx.Process(target=_worker, args=(r, world, port, a, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = dict(gather(procs, q, world, timeout=900))
        for p in procs:
            p.join(timeout=60)
        for r, v in res.items():
            if isinstance(v, str):
                print(v, file=sys.stderr)
                sys.exit(1)
        o = res[0]
        print(json.dumps({"world": world, "dtype": a.dtype, "batch_total": a.batch, "batch_per_rank": a.batch // world,
                          "ms_per_step": o["ms_per_step"], "value_seq_s": o["value"], "allreduce": o["allreduce"],
                          "buckets": o["buckets"], "allreduce_exposed_ms_per_step": o["allreduce_exposed_ms_per_step"],
                          "losses_finite": o["losses_finite"], "peak_mem_gb_rank0": o["peak_mem_gb_rank0"]}),
              flush=True)


if __name__ == "__main__":
    main()
