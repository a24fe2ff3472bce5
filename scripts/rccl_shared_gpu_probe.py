"""Probe: can two RCCL ranks share ONE GPU (the gpurun boxes have one MI355X)?

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 scripts/rccl_shared_gpu_probe.py

Each rank binds cuda:0, initialises the nccl (= RCCL) backend, all-reduces a rank-valued tensor and
prints the result.  NCCL-style libraries usually refuse two ranks on one device ("duplicate GPU");
if RCCL accepts it, multi-rank GradSync / GraphedStep runs become testable on a one-GPU box.
"""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.full((1 << 20,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        ok = bool((x == world * (world + 1) / 2).all())
        print(json.dumps({"rank": rank, "world": world, "all_reduce_ok": ok, "value": float(x[0])}), flush=True)
        dist.destroy_process_group()
        return 0 if ok else 1
    except Exception as e:  # noqa: BLE001 -- report what RCCL said
        print(json.dumps({"rank": rank, "error": repr(e)[:500]}), flush=True)
        return 3


if __name__ == "__main__":
    sys.exit(main())
