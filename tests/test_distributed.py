"""Data-parallel correctness on CPU (gloo, world_size 2) — SURVEY §4 item 3.

* bucketed DP gradients (two buckets per model, each all-reduce launched from the reverse pass as
  soon as its layers are final) equal the single-process gradient of the concatenated global
  batch (fp64), for the GP critic and the generator;
* a DP training run keeps every rank's parameters bit-identical (same averaged update everywhere).
The same code path runs over RCCL on GPUs (backend 'nccl'); only the backend differs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from _spawn import gather


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import hfrep  # noqa: F401
        from hfrep.parallel.dp import GradSync, init_distributed
        from hfrep.train.gan_trainer import GANConfig, GANTrainer

        r, _, w, pg = init_distributed(backend="gloo")
        T, F, B = 6, 4, 8
        ds = np.random.RandomState(0).rand(30, T, F)
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=T, features=F, batch_size=B // w, hidden=8,
                        dtype="float64")
        tr = GANTrainer(cfg, ds, process_group=pg, rank=r, world=w, param_dtype=torch.float64)
        g = torch.Generator().manual_seed(5)
        real = torch.rand(B, T, F, generator=g, dtype=torch.float64)
        noise = torch.randn(B, T, F, generator=g, dtype=torch.float64)
        alpha = torch.rand(B, generator=g, dtype=torch.float64)
        sl = slice(r * (B // w), (r + 1) * (B // w))
        with torch.no_grad():
            fake = tr.generator.predict(noise)
            tr.critic_gp_grads(real[sl], fake[sl], alpha[sl])  # launches its bucket all-reduces
            tr._sync(tr.critic)                                # ... and waits for them
            tr.generator_grads(noise[sl])
            tr._sync(tr.generator)
        out = {"critic": tr.critic.flat.grad.clone(), "gen": tr.generator.flat.grad.clone()}
        tr.critic.zero_grad(); tr.generator.zero_grad()
        tr.train(3, verbose=False)
        out["params"] = torch.cat([tr.generator.flat.detach(), tr.critic.flat.detach()])
        q.put((r, {k: v.numpy() for k, v in out.items()}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback

        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gloo_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r, v in gather(procs, q, world, timeout=300):
        assert not isinstance(v, str), v
        res[r] = v

    # single-process reference on the full global batch
    import hfrep  # noqa: F401
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    T, F, B = 6, 4, 8
    ds = np.random.RandomState(0).rand(30, T, F)
    cfg = GANConfig(arch="lstm", loss="wgan_gp", window=T, features=F, batch_size=B, hidden=8, dtype="float64")
    tr = GANTrainer(cfg, ds, param_dtype=torch.float64)
    g = torch.Generator().manual_seed(5)
    real = torch.rand(B, T, F, generator=g, dtype=torch.float64)
    noise = torch.randn(B, T, F, generator=g, dtype=torch.float64)
    alpha = torch.rand(B, generator=g, dtype=torch.float64)
    with torch.no_grad():
        fake = tr.generator.predict(noise)
        tr.critic_gp_grads(real, fake, alpha)
        tr.generator_grads(noise)
    np.testing.assert_allclose(res[0]["critic"], tr.critic.flat.grad.numpy(), rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(res[0]["gen"], tr.generator.flat.grad.numpy(), rtol=1e-10, atol=1e-13)
    for r in range(1, world):
        np.testing.assert_array_equal(res[0]["critic"], res[r]["critic"])
        # after DP training every rank holds identical parameters
        np.testing.assert_array_equal(res[0]["params"], res[r]["params"])


def _runner_worker(rank, world, port, ckdir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import hfrep  # noqa: F401
        from hfrep.parallel.dp import init_distributed
        from hfrep.train.gan_trainer import GANConfig, GANTrainer
        from hfrep.train.runner import RunOptions, run

        r, _, w, pg = init_distributed(backend="gloo")
        ds = np.random.RandomState(0).rand(30, 6, 4)

        def trainer():
            cfg = GANConfig(arch="lstm", loss="wgan_gp", window=6, features=4, batch_size=4, hidden=8, dtype="float64")
            return GANTrainer(cfg, ds, process_group=pg, rank=r, world=w, param_dtype=torch.float64)

        a = trainer()
        recs = run(a, RunOptions(epochs=4, log_every=1, echo=False, ckpt_dir=ckdir, ckpt_every=2))
        # a second job resumes from the newest checkpoint; rank 0 resolves the path for everyone
        b = trainer()
        recs_b = run(b, RunOptions(epochs=6, log_every=1, echo=False, ckpt_dir=ckdir, ckpt_every=2, resume="auto"))
        losses = [[x["d_loss"], x["g_loss"], x["gp"]] for x in recs]
        local = [float(v) for v in a._d_acc.reshape(-1).tolist()]
        q.put((r, {"losses": losses, "resumed_at": [x["iteration"] for x in recs_b][0], "local_last": local,
                   "params": torch.cat([b.generator.flat.detach(), b.critic.flat.detach()]).numpy()}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def test_dp_runner_averages_logged_losses_and_resumes_consistently(tmp_path):
    """C5: logged losses are the all-rank average (identical on every rank, != a rank's local
    value); resume='auto' resolves one checkpoint on rank 0 for all ranks, after a barrier that
    follows every checkpoint write."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_runner_worker, args=(r, world, port, str(tmp_path / "ck"), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r, v in gather(procs, q, world, timeout=300):
        assert not isinstance(v, str), v
        res[r] = v
    assert res[0]["losses"] == res[1]["losses"]
    last = res[0]["losses"][-1][0]
    mean_local = 0.5 * (res[0]["local_last"][0] + res[1]["local_last"][0])
    assert abs(last - mean_local) < 1e-6 * max(1.0, abs(mean_local))  # (logged through fp32 snapshots)
    assert res[0]["local_last"][0] != res[1]["local_last"][0]
    assert res[0]["resumed_at"] == res[1]["resumed_at"] == 5
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])


def _local_ckpt_worker(rank, world, port, base, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import hfrep  # noqa: F401
        from hfrep.parallel.dp import init_distributed
        from hfrep.train.gan_trainer import GANConfig, GANTrainer
        from hfrep.train.runner import RunOptions, run

        r, _, w, pg = init_distributed(backend="gloo")
        ds = np.random.RandomState(0).rand(30, 6, 4)
        ckdir = os.path.join(base, f"rank{r}")  # rank-LOCAL: only rank 0's directory gets files

        def trainer():
            cfg = GANConfig(arch="lstm", loss="wgan_gp", window=6, features=4, batch_size=4, hidden=8, dtype="float64")
            return GANTrainer(cfg, ds, process_group=pg, rank=r, world=w, param_dtype=torch.float64)

        full = trainer()
        run(full, RunOptions(epochs=6, log_every=1, echo=False))
        a = trainer()
        run(a, RunOptions(epochs=4, log_every=1, echo=False, ckpt_dir=ckdir, ckpt_every=4))
        b = trainer()
        recs = run(b, RunOptions(epochs=6, log_every=1, echo=False, ckpt_dir=ckdir, resume="auto"))
        q.put((r, {"resumed_at": recs[0]["iteration"], "files": sorted(os.listdir(ckdir)) if os.path.isdir(ckdir) else [],
                   "params": torch.cat([b.generator.flat.detach(), b.critic.flat.detach()]).numpy(),
                   "full": torch.cat([full.generator.flat.detach(), full.critic.flat.detach()]).numpy()}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def test_dp_resume_from_rank_local_checkpoint_dir(tmp_path):
    """ckpt_dir visible to rank 0 only: rank 0 reads the state and broadcasts it; the resumed run
    continues bitwise like an uninterrupted one on every rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_ckpt_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r, v in gather(procs, q, world, timeout=300):
        assert not isinstance(v, str), v
        res[r] = v
    assert res[1]["files"] == [] and res[0]["files"]
    assert res[0]["resumed_at"] == res[1]["resumed_at"] == 5
    for r in range(world):
        np.testing.assert_array_equal(res[r]["params"], res[r]["full"])


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import argparse
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        import hfrep  # noqa: F401
        from hfrep.parallel.dp import init_distributed

        r, _, w, pg = init_distributed(backend="gloo")
        args = argparse.Namespace(window=6, features=4, batch_per_gpu=4, hidden=8, model="mtss_wgan_gp",
                                  dataset_windows=32, warmup=1, steps=2, trace_out="", profile_steps=0)
        if r == world - 1:  # the slowest rank sets the job's elapsed time
            import time

            orig = bench.time.perf_counter
            calls = {"n": 0}

            def slow():
                calls["n"] += 1
                return orig() + (0.5 if calls["n"] == 2 else 0.0)  # +0.5 s on the timed window's end

            bench.time = type("T", (), {"perf_counter": staticmethod(slow)})
        out = bench._measure(args, "float32", r, w, pg, torch.device("cpu"))
        q.put((r, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def test_bench_aggregate_uses_max_elapsed_over_ranks():
    """bench.py at world 8 (gloo, CPU, tiny shape): every rank reports the same elapsed time, the
    MAX of the per-rank timed windows, and value = all ranks' windows x steps / that time."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r, v in gather(procs, q, world, timeout=300):
        assert not isinstance(v, str), v
        res[r] = v
    local = [res[r]["elapsed_local_s"] for r in range(world)]
    assert local[world - 1] >= 0.5 and local[world - 1] == max(local)
    for r in range(world):
        assert res[r]["elapsed_s"] == max(local)
        per_rank_windows = 5 * 4 + 4  # n_critic * B + B
        assert res[r]["windows_per_step"] == per_rank_windows * world
        assert res[r]["value"] == round(per_rank_windows * world * 2 / max(local), 2)
        # the DP fields of the record: gloo buckets (no GPU events: zero exposed wait), one entry per rank
        assert res[r]["allreduce"] == "gloo" and res[r]["buckets"] == 2
        assert res[r]["allreduce_exposed_ms_per_step"] == [0.0] * world
        # the job as the process group saw it, and the bytes each rank reduces per step
        assert res[r]["world_pg"] == world and res[r]["rank_devices"] == ["cpu"] * world
        assert res[r]["allreduce_bytes_per_step"] > 0 and res[r]["allreduce_bytes_per_step"] % 4 == 0


def test_bench_torchrun_world8_record_shape():
    """``torchrun --nproc-per-node 8 bench.py --gpus 8`` as the driver launches it (gloo on the CPU):
    rank 0 prints ONE JSON line naming the 8-rank job -- n_gpus, world_pg, 8 rank devices, dp8, the
    aggregate over all ranks and the all-reduce bytes of the MTSS-WGAN-GP step."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "8", "--steps", "1",
           "--warmup", "0", "--batch-per-gpu", "4", "--window", "6", "--features", "3", "--dataset-windows", "16",
           "--dtype", "float32"]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["world_pg"] == 8 and len(rec["rank_devices"]) == 8
    assert rec["config"]["parallelism"] == "dp8" and rec["config"]["global_batch"] == 32
    assert rec["config"]["windows_per_step"] == 8 * (5 * 4 + 4) and rec["steps"] == 1 and rec["warmup"] == 0
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["allreduce"] == "gloo"
    # critic buffer 5 times + generator once, fp32
    assert rec["allreduce_bytes_per_step"] > 0 and len(rec["allreduce_exposed_ms_per_step"]) == 8


def test_gradsync_graph_routes():
    """What a hipGraph capture may contain follows the routes the eager buckets took: a bucket
    that fell back from P2P to gloo makes the step uncapturable; one that fell back to RCCL needs the
    capture-only communicator; all-P2P needs neither."""
    from hfrep.parallel.dp import GradSync

    gs = GradSync(None, 2)
    gs.use_p2p, gs.backend, gs.group = True, "nccl", object()
    assert gs.needs_graph_group()  # no eager step seen yet: switch (safe)
    gs.routes = {"p2p"}
    assert not gs.needs_graph_group() and gs.graph_capturable()
    gs.routes = {"p2p", "rccl"}  # a bucket over HFREP_DP_P2P_CAP went to RCCL
    assert gs.needs_graph_group() and gs.graph_capturable()
    gs.backend = "gloo"
    gs.routes = {"p2p", "gloo"}  # forced P2P on a gloo group, an oversize bucket took gloo
    assert not gs.graph_capturable() and not gs.needs_graph_group()
    gs.routes = {"p2p"}
    assert gs.graph_capturable()
    assert GradSync(None, 1).graph_capturable()


def test_bench_refuses_gpus_world_mismatch():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr


def test_nccl_graph_safe_env_defaults(monkeypatch):
    """RCCL collectives captured into hipGraphs need ProcessGroupNCCL's event cache off (a captured
    collective could re-record a cached event the watchdog still polls: hipErrorCapturedEvent); the
    default is set, an explicit user setting wins."""
    from hfrep.parallel.dp import nccl_graph_safe_env

    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    nccl_graph_safe_env()
    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "0"
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")
    nccl_graph_safe_env()
    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "1"


def test_gradsync_p2p_selection(monkeypatch):
    """HFREP_DP_P2P=1 routes fp32 GPU buckets of <= HFREP_DP_P2P_CAP floats to the one-shot IPC
    all-reduce (parallel/p2p.py) -- only for RCCL groups of > 1 rank; everything else stays on the
    process group's collective (the kernel itself: tests/test_p2p_gpu.py)."""
    from hfrep.parallel.dp import GradSync

    monkeypatch.setenv("HFREP_DP_P2P", "1")
    monkeypatch.setenv("HFREP_DP_P2P_CAP", "1000")
    gs = GradSync(None, 2)
    assert not gs.use_p2p  # no nccl group
    gs.use_p2p = True
    assert gs.p2p_cap == 1000
    assert gs._p2p_for(torch.zeros(10)) is None  # CPU tensor
    assert gs._p2p_for(torch.zeros(2000)) is None  # over the cap
    monkeypatch.setenv("HFREP_DP_P2P", "force")  # any group carries the handles (shared-GPU benches)
    assert GradSync(None, 2).use_p2p and not GradSync(None, 1).use_p2p
    assert GradSync(None, 2).graph_capturable()
    monkeypatch.delenv("HFREP_DP_P2P")
    assert not GradSync(None, 2).use_p2p
    assert not GradSync(None, 2).graph_capturable()  # gloo buckets cannot be captured
    gs = GradSync(None, 2)
    assert gs.exposed_wait_ms() == 0.0 and gs.check_errors() is None and gs.close() is None
