"""The one-shot IPC all-reduce (``csrc/p2p.hip``, ``parallel/p2p.py``) with 2 and 8 real processes.

RCCL refuses two ranks on one GPU (``profiles/r04_main/rccl_shared_gpu_probe.txt``), but HIP IPC does
not: 2 (and 8, the node's rank count) spawned processes all bind cuda:0, exchange their buffers' IPC
handles over a gloo group, and run the same kernel that would read the peers' buffers over xGMI on a
node.  Checks: every size (1 element to the capacity, vector and scalar tails) equals the fp32
rank-order sum bit for bit on every rank, the average variant, a hipGraph-captured call replayed with new inputs (device-side
epochs), GradSync's bucketed start_ / finish_ through the side stream, and a clean error word; and
the failure path: a peer that skips a call makes the other rank give up after the wall-clock timeout
with NaN (never a finite stale result), and both ranks raise P2PTimeout.
"""
import os
import socket
import traceback

import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 3, 4, 1000, 4097, 65538, 1 << 20]


def _inputs(n, tag, world):
    import torch

    out = []
    for r in range(world):
        g = torch.Generator().manual_seed(1000003 * n + 7919 * tag + r)
        out.append(torch.randn(n, generator=g))
    return out


def _expect(xs, scale=None):
    s = xs[0] * 0
    for x in xs:
        s = s + x  # fp32, rank order: the kernel's summation
    return s if scale is None else s * scale


def _worker(rank, world, port, q):
    try:
        import os

        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.parallel.dp import GradSync
        from hfrep.parallel.p2p import P2PAllReduce

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ar = P2PAllReduce(dist.group.WORLD, cap=1 << 20, device=dev)
        res = {"rank": rank, "bad": []}
        tag = 0
        for n in SIZES:
            for avg in (False, True):
                tag += 1
                xs = _inputs(n, tag, world)
                x = xs[rank].to(dev)
                dist.barrier()
                ar.all_reduce_(x, average=avg)
                torch.cuda.synchronize()
                if not torch.equal(x.cpu(), _expect(xs, torch.tensor(1.0 / world) if avg else None)):
                    res["bad"].append(("eager", n, avg))
        # hipGraph: capture once, replay with new inputs
        n = 70001
        xst = torch.zeros(n, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.barrier()
            ar.all_reduce_(xst)  # eager warmup on the capture stream
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ar.all_reduce_(xst)
        for rep in range(3):
            tag += 1
            xs = _inputs(n, tag, world)
            xst.copy_(xs[rank].to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            if not torch.equal(xst.cpu(), _expect(xs)):
                res["bad"].append(("graph", rep))
        # GradSync's bucketed path (start_ on the side stream, finish_ joins it)
        gs = GradSync(dist.group.WORLD, world, buckets=2)
        gs.use_p2p = True  # (the env switch is for nccl groups; the handles here go over gloo)
        tag += 1
        xs = _inputs(50000, tag, world)
        flat = xs[rank].to(dev)
        dist.barrier()
        gs.start_(flat[:20000])
        gs.start_(flat[20000:])
        gs.finish_()
        torch.cuda.synchronize()
        want = torch.cat([_expect([x[:20000] for x in xs], torch.tensor(1.0 / world)),
                          _expect([x[20000:] for x in xs], torch.tensor(1.0 / world))])
        if not torch.equal(flat.cpu(), want):
            res["bad"].append(("gradsync",))
        ar.check()
        res["epochs"] = int(ar.buf[:4].view(torch.int32).item())
        dist.barrier()
        ar.close()
        gs.p2p.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        q.put(traceback.format_exc())


# (8 ranks on one GPU spawn 8 interpreters that each import torch + the native library: minutes on a
# cold box, so that size runs on request, HFREP_TEST_P2P_WORLD8=1; profiles/r04_p2p has its runs)
@pytest.mark.parametrize("world", [2, 4] + ([8] if os.environ.get("HFREP_TEST_P2P_WORLD8") == "1" else []))
def test_p2p_allreduce_processes(cuda, world):
    import torch.multiprocessing as mp

    from _spawn import gather

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = gather(procs, q, world, timeout=240)
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert not isinstance(r, str), r
        assert r["bad"] == [], r
        # 14 eager + 1 warmup + 3 replays
        assert r["epochs"] == 2 * len(SIZES) + 1 + 3, r


def _dp_worker(rank, world, port, q):
    """Data-parallel MTSS-WGAN-GP training (fp32, native kernels) with the gradient buckets averaged
    by the one-shot IPC all-reduce; every rank on cuda:0, gloo for the scalars / broadcast."""
    try:
        import os

        import numpy as np
        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.train.gan_trainer import GANConfig, GANTrainer

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ds = np.random.RandomState(0).rand(512, 24, 32).astype(np.float32)
        B = 128
        cfg = dict(arch="lstm", loss="wgan_gp", window=24, features=32, dtype="float32")
        tr = GANTrainer(GANConfig(batch_size=B // world, **cfg), ds, device=dev, process_group=dist.group.WORLD,
                        rank=rank, world=world)
        tr.grad_sync.use_p2p = True  # (the env switch is for nccl groups)
        g = torch.Generator().manual_seed(5)
        real = torch.rand(B, 24, 32, generator=g).to(dev)
        noise = torch.randn(B, 24, 32, generator=g).to(dev)
        alpha = torch.rand(B, generator=g).to(dev)
        sl = slice(rank * (B // world), (rank + 1) * (B // world))
        with torch.no_grad():
            fake = tr.generator.predict(noise)
            tr.critic_gp_grads(real[sl], fake[sl], alpha[sl])
            tr._sync(tr.critic)
        dp_grad = tr.critic.flat.grad.detach().clone()
        used_p2p = tr.grad_sync.p2p is not None
        # the same gradient from one process on the whole batch
        ref = GANTrainer(GANConfig(batch_size=B, **cfg), ds, device=dev)
        ref.generator.flat.data.copy_(tr.generator.flat.data)
        ref.critic.flat.data.copy_(tr.critic.flat.data)
        with torch.no_grad():
            ref.critic_gp_grads(real, ref.generator.predict(noise), alpha)
        full = ref.critic.flat.grad.detach()
        rel = float((dp_grad - full).norm() / full.norm())
        tr.critic.zero_grad()
        tr.generator.zero_grad()
        tr.train(3, verbose=False)
        torch.cuda.synchronize()
        params = torch.cat([tr.generator.flat.detach(), tr.critic.flat.detach()]).cpu()
        tr.grad_sync.p2p.check()
        dist.barrier()
        tr.grad_sync.p2p.close()
        dist.destroy_process_group()
        q.put({"rank": rank, "rel": rel, "p2p": used_p2p, "params": params.numpy(),
               "finite": bool(torch.isfinite(params).all())})
    except Exception:
        q.put(traceback.format_exc())


def test_dp_training_over_p2p_allreduce(cuda):
    import numpy as np
    import torch.multiprocessing as mp

    from _spawn import gather

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = gather(procs, q, 2, timeout=240)
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert not isinstance(r, str), r
        assert r["p2p"] and r["finite"], r
        # the averaged half-batch gradients = the full-batch gradient up to fp32 summation order
        assert r["rel"] < 1e-5, r["rel"]
    # identical bits on every rank after three DP iterations
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])


def _timeout_worker(rank, port, q):
    """Rank 1 skips one call: rank 0's call must give up after its timeout, return NaN (not a finite
    stale gradient) and raise; rank 1's next call must see the poison at once and raise too."""
    try:
        import os
        import time

        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.parallel.p2p import P2PAllReduce, P2PTimeout

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ar = P2PAllReduce(dist.group.WORLD, cap=1 << 16, device=dev, timeout_s=2.0)
        res = {"rank": rank}
        x = torch.full((5000,), float(rank + 1), device=dev)
        dist.barrier()
        ar.all_reduce_(x)  # a good call first
        torch.cuda.synchronize()
        res["first_ok"] = bool((x == 3.0).all())
        ar.check()
        dist.barrier()
        if rank == 0:
            y = torch.ones(5000, device=dev)
            ar.poll()  # snapshot before the failing call: clean
            t0 = time.perf_counter()
            ar.all_reduce_(y)  # rank 1 never joins this one
            torch.cuda.synchronize()
            res["wait_s"] = time.perf_counter() - t0
            res["nan"] = bool(torch.isnan(y).all())
            try:
                ar.poll()  # lands the clean snapshot, takes a new one
                torch.cuda.synchronize()
                ar.poll()  # the new snapshot holds the error word
                res["poll_raised"] = False
            except P2PTimeout:
                res["poll_raised"] = True
            res["epochs"] = int(ar.buf[:4].view(torch.int32).item())
        dist.barrier()  # rank 1 stays alive (its buffer mapped) until rank 0 has given up
        if rank == 1:
            z = torch.ones(5000, device=dev)
            t0 = time.perf_counter()
            ar.all_reduce_(z)  # poisoned by rank 0: NaN without waiting
            torch.cuda.synchronize()
            res["wait_s"] = time.perf_counter() - t0
            res["nan"] = bool(torch.isnan(z).all())
        try:
            ar.check()
            res["check_raised"] = False
        except P2PTimeout as e:
            res["check_raised"] = True
            res["msg"] = str(e)
        ar.close()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        q.put(traceback.format_exc())


def test_p2p_allreduce_missing_peer_fails_loud(cuda):
    import torch.multiprocessing as mp

    from _spawn import gather

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_timeout_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = gather(procs, q, 2, timeout=180)
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert not isinstance(r, str), r
        assert r["first_ok"] and r["nan"] and r["check_raised"], r
        assert "rank 0 gave up" in r["msg"], r
    r0 = [r for r in res if r["rank"] == 0][0]
    r1 = [r for r in res if r["rank"] == 1][0]
    assert 1.5 < r0["wait_s"] < 30, r0  # the time bound, not a poll count
    assert r0["poll_raised"], r0
    assert r0["epochs"] == 1, r0  # the failed call did not advance the epoch
    assert r1["wait_s"] < 1.0, r1  # poisoned: no wait


def _graph_worker(rank, world, port, q):
    """A hipGraph-replayed DP training step whose gradient buckets go through the P2P all-reduce, against
    the eager step of an identical trainer: bitwise equal parameters after 5 iterations, on every rank."""
    try:
        import os

        import numpy as np
        import torch
        import torch.distributed as dist

        import hfrep  # noqa: F401
        from hfrep.train.gan_trainer import GANConfig, GANTrainer
        from hfrep.train.runner import GraphedStep

        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        os.environ["HFREP_GRAPH_DP"] = "1"  # captured DP collectives are opt-in
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ds = np.random.RandomState(0).rand(512, 24, 32).astype(np.float32)
        cfg = GANConfig(arch="lstm", loss="wgan_gp", window=24, features=32, batch_size=64, dtype="float32")
        trs = []
        for _ in range(2):
            tr = GANTrainer(cfg, ds, device=dev, process_group=dist.group.WORLD, rank=rank, world=world)
            tr.grad_sync.use_p2p = True  # (the env switch is for nccl groups; the handles go over gloo)
            trs.append(tr)
        graphed, eager = trs
        step = GraphedStep(graphed, warmup=2)
        for _ in range(5):
            step()
            eager.train_step()
        torch.cuda.synchronize()
        pg = torch.cat([graphed.generator.flat.detach(), graphed.critic.flat.detach()]).cpu()
        pe = torch.cat([eager.generator.flat.detach(), eager.critic.flat.detach()]).cpu()
        res = {"rank": rank, "captured": step.graph is not None, "same": bool(torch.equal(pg, pe)),
               "finite": bool(torch.isfinite(pg).all()), "params": pg.numpy(),
               "second_comm": graphed.grad_sync._graph_group is not None}
        for tr in trs:
            tr.grad_sync.check_errors(blocking=True)
            tr.close()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        q.put(traceback.format_exc())


def test_graphed_dp_step_over_p2p(cuda):
    import numpy as np
    import torch.multiprocessing as mp

    from _spawn import gather

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = gather(procs, q, 2, timeout=240)
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert not isinstance(r, str), r
        assert r["captured"] and r["same"] and r["finite"], {k: v for k, v in r.items() if k != "params"}
        assert not r["second_comm"], r["rank"]  # P2P buckets: no second (graph-only) communicator
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])
