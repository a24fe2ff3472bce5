"""The RCCL (``nccl`` backend) branch of the data-parallel gradient sync on real hardware.

One GPU cannot host two RCCL ranks, so a 1-rank RCCL group stands in: ``GradSync`` is told the
job has 2 ranks, which sends every gradient bucket through ``all_reduce(AVG)`` on the nccl
backend (the async, reverse-pass-overlapped ``start_`` / ``finish_`` path of parallel/dp.py);
AVG over the one real member is exact, so the trainer must stay bitwise equal to a trainer with
no sync at all.  The second test captures the same step, collectives included, into a hipGraph
(train/runner.py GraphedStep; opt-in under DP with HFREP_GRAPH_DP=1 until a >= 2-GPU run pins it).  Both run in a spawned process so the
process group never leaks into other tests.
"""
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(port, graph, key, q):
    try:
        import os

        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.parallel.dp import GradSync
        from hfrep.train.gan_trainer import GANConfig, GANTrainer
        from hfrep.train.runner import GraphedStep

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        from hfrep.parallel.dp import nccl_graph_safe_env

        nccl_graph_safe_env()  # (before the process group: RCCL events are not recycled into captures)
        os.environ["HFREP_GRAPH_DP"] = "1"  # captured DP collectives are opt-in
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        ds = np.random.RandomState(0).rand(256, 24, 32).astype(np.float32)
        cfg = dict(arch=key[0], loss=key[1], window=24, features=32, batch_size=64, dtype="float32")
        ref = GANTrainer(GANConfig(**cfg), ds, device=dev)
        syn = GANTrainer(GANConfig(**cfg), ds, device=dev)
        syn.grad_sync = GradSync(dist.group.WORLD, 2, buckets=2)
        assert syn.grad_sync.backend == "nccl"
        step = GraphedStep(syn, warmup=2) if graph else syn.train_step
        for _ in range(5):
            ref.train_step()
            step()
        torch.cuda.synchronize()
        out = dict(g=torch.equal(ref.generator.flat, syn.generator.flat),
                   c=torch.equal(ref.critic.flat, syn.critic.flat),
                   finite=bool(torch.isfinite(syn.critic.flat).all()),
                   captured=bool(graph and step.graph is not None))
        dist.destroy_process_group()
        q.put(out)
    except Exception:
        q.put(traceback.format_exc())


def _run(graph, key=("lstm", "wgan_gp")):
    import torch.multiprocessing as mp

    from _spawn import gather

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, graph, key, q))
    p.start()
    (res,) = gather([p], q, 1, timeout=240)  # a dead child fails within seconds, with its exit code
    assert not isinstance(res, str), res
    return res


def test_rccl_bucketed_grad_sync(cuda):
    res = _run(graph=False)
    assert res["g"] and res["c"] and res["finite"], res


# BASELINE configs 3-5: the vanilla MLP GAN, the MLP WGAN-GP and the LSTM WGAN-GP
@pytest.mark.parametrize("key", [("lstm", "wgan_gp"), ("mlp", "wgan_gp"), ("mlp", "gan")])
def test_rccl_grad_sync_in_graph(cuda, key):
    res = _run(graph=True, key=key)
    assert res["captured"] and res["g"] and res["c"] and res["finite"], res
