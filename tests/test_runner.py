"""Run driver: JSONL logging, checkpoint/resume after an injected fault, NaN guard, CLI (CPU).

SURVEY.md §5: the reference saves only the final generator, so a crash loses the run; here the
resumed run must continue bitwise-identically (fp32 on CPU) from the newest checkpoint.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import hfrep  # noqa: F401
from hfrep.data.windows import synthetic_windows
from hfrep.train.gan_trainer import GANConfig, GANTrainer
from hfrep.train.runner import InjectedFault, NonFiniteLoss, RunOptions, latest_checkpoint, run
from hfrep.utils.logger import read_jsonl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trainer(arch="lstm", loss="wgan_gp"):
    ds = synthetic_windows(64, 12, 6, seed=3)
    cfg = GANConfig(arch=arch, loss=loss, window=12, features=6, batch_size=8, hidden=16, seed=5, log_every=1)
    return GANTrainer(cfg, ds)


@pytest.mark.parametrize("key", [("lstm", "wgan_gp"), ("mlp", "wgan"), ("lstm", "gan")])
def test_resume_after_fault_is_bitwise(tmp_path, key):
    clean = _trainer(*key)
    run(clean, RunOptions(epochs=6, log_every=2, echo=False))

    ck = str(tmp_path / "ck")
    a = _trainer(*key)
    with pytest.raises(InjectedFault):
        run(a, RunOptions(epochs=6, log_every=2, echo=False, ckpt_dir=ck, ckpt_every=2, fault_at=5))
    assert latest_checkpoint(ck).endswith("state_000000004.pt")
    b = _trainer(*key)  # a fresh process would start from the same seed-initialised state
    recs = run(b, RunOptions(epochs=6, log_every=1, echo=False, ckpt_dir=ck, resume="auto"))
    assert b.iteration == 6 and [r["iteration"] for r in recs] == [5, 6]
    assert torch.equal(b.generator.flat, clean.generator.flat)
    assert torch.equal(b.critic.flat, clean.critic.flat)
    assert torch.equal(b.opt.iterations, clean.opt.iterations)


def test_checkpoint_rotation(tmp_path):
    t = _trainer()
    run(t, RunOptions(epochs=5, log_every=5, echo=False, ckpt_dir=str(tmp_path), ckpt_every=1, keep=2))
    files = sorted(os.listdir(tmp_path))
    assert files == ["state_000000004.pt", "state_000000005.pt"]


def test_jsonl_log_records(tmp_path):
    t = _trainer()
    log = str(tmp_path / "run.jsonl")
    recs = run(t, RunOptions(epochs=4, log_every=2, echo=False, log_path=log))
    rows = read_jsonl(log)
    assert [r["iteration"] for r in rows] == [2, 4] == [r["iteration"] for r in recs]
    for r in rows:
        for k in ("d_loss", "d_real", "d_fake", "gp", "g_loss", "windows_per_s"):
            assert np.isfinite(r[k])
        assert abs(r["d_loss"] - (r["d_real"] + r["d_fake"] + 10.0 * r["gp"])) < 1e-4 * max(1.0, abs(r["d_loss"]))


def test_nan_guard_stops_the_run():
    t = _trainer()
    with torch.no_grad():
        t.critic.flat[:5] = float("nan")
    with pytest.raises(NonFiniteLoss):
        run(t, RunOptions(epochs=10, log_every=1, echo=False))
    assert t.iteration <= 3  # detected within one deferred log interval


def test_env_fault_hook(monkeypatch):
    monkeypatch.setenv("HFREP_FAULT_AT", "2:0")
    t = _trainer()
    with pytest.raises(InjectedFault):
        run(t, RunOptions(epochs=5, log_every=1, echo=False))
    assert t.iteration == 2


def test_cli_train_generate_eval(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    py = [sys.executable, "-m", "hfrep"]
    gen_dir = tmp_path / "gen"
    out = subprocess.run(py + ["train", "--preset", "smoke", "--epochs", "2", "--batch-size", "8", "--n-windows", "64",
                               "--window", "12", "--features", "6", "--quiet", "--device", "cpu",
                               "--save-dir", str(gen_dir), "--log", str(tmp_path / "l.jsonl")],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    saved = json.loads(out.stdout.strip().splitlines()[-1])["saved"]
    assert os.path.exists(saved) and os.path.basename(saved).startswith("MTSS_GAN_GP")
    fake = tmp_path / "fake.npy"
    out = subprocess.run(py + ["generate", "--ckpt", saved, "--n", "32", "--device", "cpu", "--out", str(fake)],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    arr = np.load(fake)
    assert arr.shape == (32, 12, 6) and np.isfinite(arr).all()
    real = tmp_path / "real.npy"
    np.save(real, synthetic_windows(32, 12, 6, seed=9))
    out = subprocess.run(py + ["eval", "--real", str(real), "--fake", str(fake), "--metrics", "wasserstein,lp_dist"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout)
    assert set(res) == {"wasserstein", "lp_dist"} and all(np.isfinite(v) for v in res.values())


def test_trace_ranges_and_profile(tmp_path):
    """Phase ranges (utils/trace.py): no-op unless enabled; profile_steps exports a Chrome trace
    whose events include the trainer's phase names."""
    import json

    import numpy as np
    import torch

    from hfrep.train.gan_trainer import GANConfig, GANTrainer
    from hfrep.utils import trace

    with trace.trange("nothing"):  # disabled: plain pass-through
        pass
    ds = np.random.RandomState(0).rand(64, 12, 8).astype(np.float32)
    tr = GANTrainer(GANConfig(arch="lstm", loss="wgan_gp", window=12, features=8, batch_size=4, dtype="float64"), ds,
                    param_dtype=torch.float64)
    out = tmp_path / "trace.json"
    table = trace.profile_steps(tr.train_step, 1, str(out))
    names = {e.get("name") for e in json.loads(out.read_text())["traceEvents"]}
    for phase in ("critic/sample", "critic/w_terms", "critic/gp_input_grad", "critic/gp_second_order", "optimizer",
                  "generator"):
        assert phase in names, phase
    assert "critic/w_terms" in table
    assert not trace.enabled()
