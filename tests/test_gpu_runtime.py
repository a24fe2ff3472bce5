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


def test_run_with_graph_and_log(cuda, tmp_path):
    t = _trainer(cuda)
    recs = run(t, RunOptions(epochs=6, log_every=2, echo=False, log_path=str(tmp_path / "r.jsonl"), graph=True))
    assert [r["iteration"] for r in recs] == [2, 4, 6]
    assert all(np.isfinite(r["d_loss"]) and np.isfinite(r["g_loss"]) for r in recs)
