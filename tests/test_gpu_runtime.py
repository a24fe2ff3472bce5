"""GPU runtime: hipGraph replay of the whole iteration, bitwise run-to-run determinism, JSONL run.

SURVEY.md §5 (race detection / determinism): two runs with the same seed must agree bitwise;
every cross-workgroup reduction in the kernel library is a fixed-order slab reduce (no float
atomics), so this holds for the bf16 flagship configuration too.
"""
import numpy as np
import pytest
import torch

import hfrep  # noqa: F401
from hfrep.data.windows import synthetic_windows
from hfrep.train.gan_trainer import GANConfig, GANTrainer
from hfrep.train.runner import GraphedStep, RunOptions, run

pytestmark = pytest.mark.gpu


def _trainer(cuda, dtype="bfloat16", key=("lstm", "wgan_gp"), B=256, T=24, F=32):
    ds = synthetic_windows(1024, T, F, seed=1)
    cfg = GANConfig(arch=key[0], loss=key[1], window=T, features=F, batch_size=B, seed=11, dtype=dtype)
    return GANTrainer(cfg, ds, device=cuda)


@pytest.mark.parametrize("key", [("lstm", "wgan_gp"), ("lstm", "wgan"), ("mlp", "gan")])
def test_determinism_bitwise(cuda, key):
    a, b = _trainer(cuda, key=key), _trainer(cuda, key=key)
    for _ in range(3):
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert torch.equal(a.generator.flat, b.generator.flat)
    assert torch.equal(a.critic.flat, b.critic.flat)
    assert torch.equal(a._d_acc, b._d_acc)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_graph_replay_matches_eager(cuda, dtype):
    eager, graphed = _trainer(cuda, dtype), _trainer(cuda, dtype)
    for _ in range(5):
        eager.train_step()
    step = GraphedStep(graphed, warmup=2)  # 2 eager steps, capture, then replays
    for _ in range(5):
        step()
    assert step.graph is not None
    torch.cuda.synchronize()
    assert graphed.iteration == eager.iteration == 5
    assert torch.equal(graphed.generator.flat, eager.generator.flat)
    assert torch.equal(graphed.critic.flat, eager.critic.flat)
    assert torch.equal(graphed._d_acc, eager._d_acc)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("shape", [(32, 48, 35), (256, 24, 32)])
@pytest.mark.parametrize("graph", [False, True])
def test_concurrent_chains_match_sequential(cuda, dtype, shape, graph):
    """Small-batch side-stream overlap (GANTrainer.concurrent: the GP input-gradient chain beside the
    W-terms chain, the next update's generator forward beside the current critic update) gives the
    sequential result bit for bit, eager and replayed from a hipGraph."""
    B, T, F = shape
    ds = synthetic_windows(1024, T, F, seed=1)
    tr = {}
    for conc in (False, True):
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=T, features=F, batch_size=B, seed=11, dtype=dtype,
                        concurrent=conc)
        t = GANTrainer(cfg, ds, device=cuda)
        assert t.concurrent == conc
        step = GraphedStep(t, warmup=2) if graph else t.train_step
        for _ in range(4):
            step()
        tr[conc] = t
    torch.cuda.synchronize()
    assert torch.equal(tr[True].generator.flat, tr[False].generator.flat)
    assert torch.equal(tr[True].critic.flat, tr[False].critic.flat)
    assert torch.equal(tr[True]._d_acc, tr[False]._d_acc)
    assert torch.equal(tr[True]._g_acc, tr[False]._g_acc)


def test_run_with_graph_and_log(cuda, tmp_path):
    t = _trainer(cuda)
    recs = run(t, RunOptions(epochs=6, log_every=2, echo=False, log_path=str(tmp_path / "r.jsonl"), graph=True))
    assert [r["iteration"] for r in recs] == [2, 4, 6]
    assert all(np.isfinite(r["d_loss"]) and np.isfinite(r["g_loss"]) for r in recs)


def _dp_worker(rank, world, port, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.parallel.dp import init_distributed

        r, _, w, pg = init_distributed(backend="gloo")  # 2 ranks share the one GPU of this box
        dev = torch.device("cuda", 0)
        ds = synthetic_windows(512, 24, 32, seed=1)
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=24, features=32, batch_size=64, seed=11, dtype="bfloat16")
        tr = GANTrainer(cfg, ds, device=dev, process_group=pg, rank=r, world=w)
        for _ in range(2):
            tr.train_step()
        torch.cuda.synchronize()
        q.put((r, torch.cat([tr.generator.flat.detach(), tr.critic.flat.detach()]).cpu().numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def test_dp_two_ranks_on_gpu_tensors(cuda):
    """The bucketed, reverse-pass-overlapped gradient sync on GPU tensors (gloo carries the
    collectives here; RCCL on a multi-GPU node): ranks stay bit-identical."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    from _spawn import gather

    res = {}
    for r, v in gather(procs, q, 2, timeout=600):
        assert not isinstance(v, str), v
        res[r] = v
    assert np.isfinite(res[0]).all()
    assert np.array_equal(res[0], res[1])


@pytest.mark.parametrize("key", [("lstm", "wgan_gp"), ("lstm", "wgan"), ("lstm", "gan"), ("mlp", "wgan_gp"),
                                 ("conv", "wgan_gp")])
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_poisoned_outputs_all_written(cuda, key, dtype):
    """Uninitialised-output detector (SURVEY.md §5 race/sanitizer row): with the debug poison mode
    every op output and workspace starts as NaN, so any element a kernel leaves unwritten (a lost
    row tile, a short store loop, a skipped padded column that is read later) turns the losses
    or gradients non-finite.  Odd batch (37) and window (23) exercise the partial-tile paths."""
    from hfrep.ops import _native

    ops = _native.native()
    prev = ops.set_debug_poison(True)
    try:
        tr = _trainer(cuda, dtype=dtype, key=key, B=37, T=23, F=32)
        for _ in range(2):
            tr.train_step()
        torch.cuda.synchronize()
        rec = tr.losses()
        assert all(np.isfinite(v) for k, v in rec.items() if k != "iteration"), rec
        for m in (tr.generator, tr.critic):
            assert bool(torch.isfinite(m.flat).all()), m.model_name
    finally:
        ops.set_debug_poison(prev)


def test_legacy_script_train_uses_graph(cuda, tmp_path):
    """The reference entry point (GAN/MTSS_WGAN_GP.py -> compat.legacy_gan WGAN_GP.train) replays
    the step from a hipGraph on the GPU; the result is bitwise the eager run's."""
    from hfrep.compat.legacy_gan import WGAN_GP

    ds = np.random.RandomState(0).rand(64, 12, 8).astype(np.float32)
    a, b = WGAN_GP(ds, device=cuda), WGAN_GP(ds, device=cuda)
    with torch.no_grad():
        b.generator.flat.copy_(a.generator.flat)
        b.critic.flat.copy_(a.critic.flat)
    ha = a.train(epochs=6, batch_size=16, save_dir=None, verbose=False, log_every=3)
    hb = b.train(epochs=6, batch_size=16, save_dir=None, verbose=False, log_every=3, graph=False)
    assert torch.equal(a.generator.flat, b.generator.flat) and torch.equal(a.critic.flat, b.critic.flat)
    assert [r["d_loss"] for r in ha] == [r["d_loss"] for r in hb]
