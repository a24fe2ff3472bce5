"""Headline benchmark: MTSS-WGAN-GP training throughput (24 x 32 windows), seq/s per node.

Metric (BASELINE.json): "seq/sec/node MTSS-WGAN-GP train (24x32 windows) at 1/2/4/8 GPUs".
One step = one reference training iteration (GAN/MTSS_WGAN_GP.py:254-287): n_critic = 5 critic
updates with the gradient penalty (second-order pass through the LSTM critic) + 1 generator update,
each followed by the fused RMSprop(5e-5) launch and — for N > 1 — an RCCL all-reduce of the flat
gradient bucket.  Windows counted per step: (n_critic * B + B) per rank; ``value`` is
the whole-job aggregate over all ranks.

Model: the reference architecture at the north-star shape — generator LSTM(100, sigmoid) -> LN ->
LSTM(100, sigmoid) -> LeakyReLU -> LN -> Dense(32); critic LSTM(100) -> LSTM(100) -> Flatten ->
Dense(1); random init; synthetic return windows (no dataset/network on the box); compute dtype
fp32 (the reference's Keras float32: fp32 storage, tapes, gradients, optimizer state and accumulation;
products on the exact-f32 MFMA or as the fp32-accurate three-term bf16 split -- each fp32 operand =
h + m + l, six of the nine products, error <= 2x the exact kernel's vs fp64,
tests/test_kernels_gpu.py test_lstmf_*split*; HFREP_FP32_EXACT=1 for exact-f32 everywhere) for the
headline record, and a bf16 sub-record
(bf16 MFMA with fp32 accumulation, fp32 master weights / optimizer) of the same config.

Usage:
    python bench.py                         # 1 GPU, defaults
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


# model -> (metric label, config description); the headline is the first one (BASELINE.json "metric")
MODELS = {
    "mtss_wgan_gp": ("seq/sec/node MTSS-WGAN-GP train (24x32 windows) at 1/2/4/8 GPUs; W-dist parity",
                     "MTSS-WGAN-GP (G: LSTM100(sigmoid)-LN-LSTM100(sigmoid)-LReLU-LN-Dense32; "
                     "C: LSTM100-LSTM100-Flatten-Dense1; GP lambda=10; n_critic=5; RMSprop 5e-5)"),
    "wgan_gp": ("seq/sec/node WGAN-GP (MLP) train (24x32 windows)",
                "WGAN-GP (G: Dense100(sigmoid)-LReLU-LN-Dense100(sigmoid)-LReLU-LN-Dense32; "
                "C: Dense100-Dense100-Flatten-Dense1; GP lambda=10; n_critic=5; RMSprop 5e-5)"),
    "gan": ("seq/sec/node vanilla GAN (MLP) train (24x32 windows)",
            "GAN (G: Dense100(sigmoid)-LReLU-LN-Dense100(sigmoid)-LReLU-LN-Dense32; "
            "D: Dense100-Dense100-Dense1(sigmoid) per step; BCE; Adam 2e-4 b1=0.5)"),
    "mtss_gan": ("seq/sec/node MTSS-GAN (LSTM) train (24x32 windows)", "MTSS-GAN (LSTM G / LSTM D, BCE, Adam)"),
    "mtss_wgan": ("seq/sec/node MTSS-WGAN (LSTM, clipped) train (24x32 windows)",
                  "MTSS-WGAN (LSTM G / LSTM-LReLU-LN critic, clip 0.01, n_critic=5, RMSprop)"),
    "conv_wgan_gp": ("seq/sec/node conv-critic WGAN-GP train (24x32 windows)",
                     "LSTM G / causal Conv1D critic, GP lambda=10, n_critic=5"),
}


def _sync(dev):
    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _device_id(dev) -> str:
    """This rank's device as the record names it: index, plus the PCI bus / UUID where the runtime exposes
    them (so an N-GPU record shows N distinct devices)."""
    import torch

    if dev.type != "cuda":
        return str(dev)
    p = torch.cuda.get_device_properties(dev)
    tags = [f"{k}={getattr(p, k)}" for k in ("pci_bus_id", "pci_device_id", "uuid") if getattr(p, k, None) is not None]
    return f"cuda:{dev.index} {p.name}" + (f" ({', '.join(str(t) for t in tags)})" if tags else "")


def _measure(args, dtype, rank, world, pg, dev):
    """Warm up, then time exactly args.steps training iterations at one compute dtype.

    The timed window is bracketed by a barrier and a device synchronisation on both sides; the
    job's elapsed time is the MAX over ranks, and ``value`` = windows per step on all ranks x steps
    / that elapsed time.  (``dev`` may be a CPU device: the gloo multi-rank test drives this path.)"""
    import numpy as np
    import torch
    import torch.distributed as dist

    from hfrep.data.windows import synthetic_windows
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    from hfrep.models import gan as zoo

    T, F, B = args.window, args.features, args.batch_per_gpu
    arch, loss = zoo.resolve(args.model)
    ds = synthetic_windows(args.dataset_windows, T, F, seed=1234)
    cfg = GANConfig(arch=arch, loss=loss, window=T, features=F, batch_size=B, dtype=dtype, seed=123,
                    hidden=getattr(args, "hidden", 100))
    tr = GANTrainer(cfg, ds, device=dev, process_group=pg, rank=rank, world=world)
    cuda = dev.type == "cuda"
    if cuda:
        torch.cuda.reset_peak_memory_stats(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        tr.train_step()
    gs = tr.grad_sync
    if gs is not None:
        gs.exposed_wait_ms()  # (drop any warmup events)
        gs.timing = True      # event pair around every bucket join of the timed steps
    _sync(dev)
    barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step()
    _sync(dev)
    barrier()
    _sync(dev)
    local = time.perf_counter() - t0
    elapsed = local
    exposed = [0.0] * world
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # each rank's exposed all-reduce wait per step: compute-stream time blocked in GradSync.finish_
        w = torch.zeros(world, dtype=torch.float64, device=dev)
        w[rank] = gs.exposed_wait_ms() / args.steps
        gs.timing = False
        dist.all_reduce(w, op=dist.ReduceOp.SUM)
        exposed = [round(float(v), 3) for v in w.cpu()]
        gs.check_errors(blocking=True)
    if args.trace_out and rank == 0:
        from hfrep.utils.trace import profile_steps

        print(profile_steps(tr.train_step, args.profile_steps or 2, args.trace_out), file=sys.stderr)
    else:
        for _ in range(args.profile_steps):
            tr.train_step()
    _sync(dev)
    losses = tr.losses()
    per_rank = tr.windows_per_iteration()
    # the job as the process group sees it: its size and every rank's device
    world_pg = dist.get_world_size(pg) if world > 1 else 1
    devices = [_device_id(dev)]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, _device_id(dev), group=pg)
    out = {
        "value": round(per_rank * world * args.steps / elapsed, 2),
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "windows_per_step": per_rank * world,
        "losses_finite": bool(all(np.isfinite(v) for k, v in losses.items() if k != "iteration")),
        "peak_mem_gb_rank0": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if cuda else 0.0,
        "elapsed_s": elapsed,
        "elapsed_local_s": local,
        "allreduce": "none" if gs is None else ("p2p" if gs.use_p2p else "rccl" if gs.backend == "nccl" else gs.backend),
        "buckets": 0 if gs is None else gs.buckets,
        "allreduce_exposed_ms_per_step": exposed,
        "world_pg": world_pg,
        "rank_devices": devices,
        # fp32 gradient bytes each rank all-reduces per step (0 on one GPU: nothing is reduced)
        "allreduce_bytes_per_step": 4 * tr.allreduce_floats_per_step() if world > 1 else 0,
    }
    tr.close()
    del tr, ds
    if cuda:
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    # per-GPU batch sized for HBM: 262144 windows per GPU use 194 GB (fp32) / 106 GB (bf16) of the 288 GB
    # (BENCH_r04.json peak_mem_gb_rank0); larger batches amortise the per-call tails of the persistent
    # kernels (profiles/r01_batch_sweep)
    ap.add_argument("--batch-per-gpu", type=int, default=262144)
    ap.add_argument("--window", type=int, default=24)
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--dtype", default="both", choices=["both", "float32", "bfloat16"],
                    help="both (default): the reference-precision fp32 record, plus a bf16 sub-record timed the "
                         "same way right after it")
    ap.add_argument("--model", default="mtss_wgan_gp", choices=sorted(MODELS),
                    help="mtss_wgan_gp (default) is the BASELINE headline; gan / wgan_gp are BASELINE configs 3 / 4 "
                         "(GAN.py, WGAN_GP.py MLP models) measured the same way")
    ap.add_argument("--dataset-windows", type=int, default=8192)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (e.g. for rocprof)")
    ap.add_argument("--trace-out", default="", help="after the timed steps: torch.profiler Chrome trace of "
                    "--profile-steps (default 2) untimed steps with the trainer's phase ranges")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import hfrep  # noqa: F401
    from hfrep.parallel.dp import env_rank, init_distributed

    _, _, env_world = env_rank()
    if env_world != args.gpus:
        # the record's n_gpus / aggregate must describe the job that actually ran
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE {env_world} (launch N > 1 with "
              f"torch.distributed.run --nproc-per-node N)", file=sys.stderr)
        sys.exit(2)
    rank, local_rank, world, pg = init_distributed()
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:  # CPU (gloo) rehearsal of the multi-rank record: tests/test_distributed.py
        dev = torch.device("cpu")

    primary = "float32" if args.dtype in ("both", "float32") else "bfloat16"
    res = _measure(args, primary, rank, world, pg, dev)
    sub = _measure(args, "bfloat16", rank, world, pg, dev) if args.dtype == "both" else None
    T, F, B = args.window, args.features, args.batch_per_gpu
    if rank == 0:
        rec = {
            "metric": MODELS[args.model][0],
            "value": res["value"],
            "unit": "seq/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # fp32 = the reference's precision (Keras float32): fp32 activations, tapes, gradients and
            # optimizer state; products on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32) or the
            # fp32-accurate three-term bf16 split (see the module docstring)
            "dtype": "fp32" if primary == "float32" else "bf16",
            "data": "synthetic",
            "config": {
                "model": MODELS[args.model][1],
                "global_batch": B * world,
                "batch_per_gpu": B,
                "seq_len": T,
                "features": F,
                "parallelism": f"dp{world}",
                "windows_per_step": res["windows_per_step"],
            },
            "losses_finite": res["losses_finite"],
            # the W-dist half of the metric is a training-quality run, not a throughput step
            "w_dist_parity": "profiles/r05_parity/README.md" if args.model == "mtss_wgan_gp" else None,
            "peak_mem_gb_rank0": res["peak_mem_gb_rank0"],
            # data-parallel gradient averaging: collective, buckets per model, and each rank's exposed
            # (non-overlapped) all-reduce wait per step
            "allreduce": res["allreduce"],
            "buckets": res["buckets"],
            "allreduce_exposed_ms_per_step": res["allreduce_exposed_ms_per_step"],
            "world_pg": res["world_pg"],
            "rank_devices": res["rank_devices"],
            "allreduce_bytes_per_step": res["allreduce_bytes_per_step"],
        }
        if sub is not None:
            # same config, same step count, timed after the fp32 run: bf16 MFMA with fp32 accumulation,
            # bf16 activations / tapes, fp32 master weights and optimizer state
            rec["bf16"] = {k: sub[k] for k in ("value", "ms_per_step", "losses_finite", "peak_mem_gb_rank0",
                                               "allreduce_exposed_ms_per_step")}
        print(json.dumps(rec))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
