"""Command-line entry points: ``python -m hfrep <command> ...`` (or ``python hfrep.py <command>``).

Commands (SURVEY.md §5 "Config / flag system"; the reference hard-codes everything per script):

  train      train any zoo model (6 reference GAN families + the conv critic variant) on the
             cleaned panel or synthetic windows, 1..N GPUs (torchrun env), JSONL log,
             periodic checkpoints, resume, NaN guard, optional hipGraph replay
  generate   generator checkpoint (.pkl/.npz/reference Keras .h5) -> (N, T, F) windows .npy
  eval       GAN_eval metric suite (GAN/GAN_eval.py:447-458 run_all) of real vs generated windows
  parity     W-dist parity: train at a preset, generate, Wasserstein vs held-out real windows
             against the real-vs-real noise floor
  clean      raw data/ -> cleaned_data/ CSVs (the reference's missing cleaning step)
  replicate  linear OLS clone benchmark (P34) and the factor-autoencoder clone (P11-P19)
  bench      the flagship throughput benchmark (bench.py contract)

Presets: ``reference`` = the scripts' constants (B=32, T=48, F=35, 5000 iterations, fp32, 1000
cleaned windows; Appendix A), ``northstar`` = the BASELINE.json config (T=24, F=32, bf16,
synthetic windows, large per-GPU batch).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

PRESETS = {
    "reference": dict(window=48, features=35, batch_size=32, epochs=5000, dtype="float32", data="cleaned",
                      n_windows=1000, seed=123, log_every=100),
    "northstar": dict(window=24, features=32, batch_size=16384, epochs=200, dtype="bfloat16", data="synthetic",
                      n_windows=65536, seed=123, log_every=20),
    "smoke": dict(window=24, features=32, batch_size=64, epochs=3, dtype="float32", data="synthetic", n_windows=512,
                  seed=123, log_every=1),
}


def _device(arg: str | None):
    import torch

    if arg:
        return torch.device(arg)
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _dataset(data: str, n: int, window: int, features: int, seed: int, rank: int = 0):
    if data == "synthetic":
        from .data.windows import synthetic_windows

        return synthetic_windows(n, window, features, seed=seed)
    if data == "cleaned":
        from .compat.legacy_gan import reference_dataset

        ds = reference_dataset(n_sample=n, window=window, seed=seed, include_rf=(features == 36))
        if ds.shape[2] != features:
            raise SystemExit(f"cleaned panel has {ds.shape[2]} features, asked for {features}")
        return ds
    if data.endswith(".npy"):
        return np.load(data, allow_pickle=False).astype(np.float32)
    raise SystemExit(f"unknown --data {data!r} (synthetic | cleaned | <windows.npy>)")


def _add_train_args(p):
    p.add_argument("--model", default="mtss_wgan_gp",
                   help="gan | wgan | wgan_gp | mtss_gan | mtss_wgan | mtss_wgan_gp | conv_wgan_gp, or a legacy "
                        "class name (GAN, WGAN, MTTS_WGAN_GP, MTTS_GAN, MTTS_WGAN, WGAN_GP)")
    p.add_argument("--preset", default="reference", choices=sorted(PRESETS))
    for k in ("window", "features", "batch_size", "epochs", "n_windows", "seed", "log_every"):
        p.add_argument("--" + k.replace("_", "-"), type=int, default=None)
    p.add_argument("--dtype", default=None, choices=["float32", "bfloat16", "float64"])
    p.add_argument("--data", default=None, help="synthetic | cleaned | path/to/windows.npy")
    p.add_argument("--lrelu-after-first", action="store_true", help="production generator variant (SURVEY Q2)")
    p.add_argument("--device", default=None)
    p.add_argument("--log", default=None, help="JSONL log path")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--ckpt-dir", default=None)
    p.add_argument("--ckpt-every", type=int, default=0)
    p.add_argument("--resume", default=None, help="checkpoint path or 'auto'")
    p.add_argument("--stop-at", type=int, default=None,
                   help="end this process at that iteration with a checkpoint in --ckpt-dir (a long run split "
                        "over several processes: rerun with --resume auto)")
    p.add_argument("--no-nan-guard", action="store_true")
    p.add_argument("--graph", action="store_true", help="replay each iteration from a captured hipGraph")
    p.add_argument("--save-dir", default="./trained_generator")
    p.add_argument("--no-save", action="store_true")
    return p


def build_trainer(a):
    """(trainer, resolved settings) for parsed ``train``/``parity`` arguments."""
    import torch

    from .models import gan as zoo
    from .parallel.dp import init_distributed
    from .train.gan_trainer import GANConfig, GANTrainer

    s = dict(PRESETS[a.preset])
    for k in s:
        v = getattr(a, k, None)
        if v is not None:
            s[k] = v
    rank, local_rank, world, pg = init_distributed()
    if a.device is None and torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    device = _device(a.device)
    arch, loss = zoo.resolve(a.model)
    cfg = GANConfig(arch=arch, loss=loss, window=s["window"], features=s["features"], batch_size=s["batch_size"],
                    epochs=s["epochs"], seed=s["seed"], dtype=s["dtype"], log_every=s["log_every"],
                    lrelu_after_first=getattr(a, "lrelu_after_first", False))
    ds = _dataset(s["data"], s["n_windows"], s["window"], s["features"], s["seed"])
    tr = GANTrainer(cfg, ds, device=device, process_group=pg, rank=rank, world=world)
    return tr, s


def _run_segment(tr, s, a):
    """Train to ``--stop-at`` (default: the preset's epochs); returns (records, finished).  An early stop
    leaves a checkpoint of that iteration in ``--ckpt-dir`` for ``--resume auto``."""
    from .train.runner import RunOptions, checkpoint_now, run

    stop = min(a.stop_at, s["epochs"]) if a.stop_at else s["epochs"]
    if stop < s["epochs"] and not a.ckpt_dir:
        raise SystemExit("--stop-at before the last iteration needs --ckpt-dir")
    graph = a.graph
    if graph and tr.world > 1 and os.environ.get("HFREP_GRAPH_DP", "0") != "1":
        # captured collectives under DP are opt-in (train/runner.py GraphedStep): step eagerly
        if tr.rank == 0:
            print("[hfrep] --graph under data parallelism needs HFREP_GRAPH_DP=1; running eager", file=sys.stderr)
        graph = False
    opts = RunOptions(epochs=stop, log_every=s["log_every"], log_path=a.log, echo=not a.quiet,
                      ckpt_dir=a.ckpt_dir, ckpt_every=a.ckpt_every, resume=a.resume, nan_guard=not a.no_nan_guard,
                      graph=graph)
    recs = run(tr, opts)
    if tr.iteration < s["epochs"]:
        checkpoint_now(tr, opts)
    tr.close()
    return recs, tr.iteration >= s["epochs"]


def cmd_train(a) -> int:
    from .utils import checkpoint

    tr, s = build_trainer(a)
    recs, done = _run_segment(tr, s, a)
    if not done:
        if tr.rank == 0:
            print(json.dumps({"partial": True, "iterations": tr.iteration, "ckpt_dir": a.ckpt_dir}))
        return 0
    if tr.rank == 0 and not a.no_save:
        prefix = tr.cfg.entry().save_prefix or "GEN"
        path = os.path.join(a.save_dir, f"{prefix}{checkpoint.timestamp()}.pkl")
        checkpoint.save_generator(path, tr.generator, dict(tr.cfg.__dict__))
        print(json.dumps({"saved": path, "iterations": tr.iteration, "last": recs[-1] if recs else None}))
    return 0


def cmd_generate(a) -> int:
    import torch

    from .utils import checkpoint
    from .utils.rng import DeviceRNG

    dev = _device(a.device)
    g, cfg = checkpoint.load_generator(a.ckpt, device=dev)
    T = a.window or cfg["window"]
    F = cfg["features"]
    rng = DeviceRNG(a.seed, dev)
    dt = torch.bfloat16 if a.dtype == "bfloat16" else torch.float32
    out = []
    with torch.no_grad():
        for s0 in range(0, a.n, a.batch):
            b = min(a.batch, a.n - s0)
            out.append(g.predict(rng.normal((b, T, F), dtype=dt)).float().cpu())
    arr = torch.cat(out).numpy()
    checkpoint.save_windows(a.out, arr)
    print(json.dumps({"out": a.out, "shape": list(arr.shape)}))
    return 0


def cmd_eval(a) -> int:
    from .eval.gan_eval import GANEval

    real = np.load(a.real, allow_pickle=False)
    fake = np.load(a.fake, allow_pickle=False)
    n = min(len(real), len(fake))
    ev = _evaluator(real[:n], fake[:n], a.name)
    if a.metrics:
        res = {m: float(np.asarray(getattr(ev, m)()).mean()) for m in a.metrics.split(",")}
    else:
        df = ev.run_all()
        res = {k: float(np.asarray(v).mean()) for k, v in df[df.columns[0]].items()}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


def _evaluator(real, fake, name="model"):
    """GANEval with the reference constructor (real, fake, dataset, subplot_title, model_name)."""
    from .eval.gan_eval import GANEval

    return GANEval(real, fake, real, [f"feature_{i}" for i in range(real.shape[-1])], [name])


def wasserstein_parity(real_train, real_holdout, fake, seed=0):
    """W-dist of generated vs held-out real windows, and the real-vs-real noise floor."""
    n = min(len(real_holdout), len(fake), len(real_train))
    w_fake = _evaluator(real_holdout[:n], fake[:n]).wasserstein()
    w_floor = _evaluator(real_holdout[:n], real_train[:n]).wasserstein()
    rs = np.random.RandomState(seed)
    # a structure-free baseline: per-feature uniform noise over the data range
    lo, hi = real_train.min(axis=(0, 1)), real_train.max(axis=(0, 1))
    unif = (lo + (hi - lo) * rs.rand(*real_holdout[:n].shape)).astype(np.float32)
    w_unif = _evaluator(real_holdout[:n], unif).wasserstein()
    return {"w_fake_vs_real": float(w_fake), "w_real_vs_real_floor": float(w_floor),
            "w_uniform_vs_real": float(w_unif), "n": int(n)}


REFERENCE_GENERATOR = "GAN/trained_generator/old/MTSS_WGAN_GP20220613_20-40-15.h5"  # 48 x 35 LSTM G (MTSS_WGAN_GP.py)


def reference_anchor(h5: str | None = None, seed: int = 123, n: int = 1000, window: int = 48, features: int = 35,
                     device="cpu"):
    """W-dist of the REFERENCE's own trained generator under the parity protocol: 1000 windows from
    N(0,1) noise (the trainer's generate() stream, seed + 7) vs the held-out real windows (seed +
    1000) of the MinMax-scaled cleaned panel, with the real-vs-real floor.  This is the number a
    reference-semantics training run should land near (GAN/GAN_eval.py:309-326; the .h5 is the
    author's MTSS-WGAN-GP generator, GAN/MTSS_WGAN_GP.py:285-287)."""
    import torch

    from .data.io import require_data_root
    from .utils import checkpoint
    from .utils.rng import DeviceRNG

    h5 = h5 or os.path.join(require_data_root(), REFERENCE_GENERATOR)
    g, _ = checkpoint.load_generator(h5, device=device)
    train = _dataset("cleaned", n, window, features, seed)
    hold = _dataset("cleaned", n, window, features, seed + 1000)
    rng = DeviceRNG(seed + 7, torch.device(device), stream=10_000)
    with torch.no_grad():
        fake = g.predict(rng.normal((n, window, features), dtype=torch.float32)).float().cpu().numpy()
    res = wasserstein_parity(train, hold, fake)
    res["generator"] = os.path.basename(h5)
    return res


def cmd_parity(a) -> int:
    import torch

    tr, s = build_trainer(a)
    _, done = _run_segment(tr, s, a)
    if tr.rank != 0:
        return 0
    if not done:
        print(json.dumps({"partial": True, "iterations": tr.iteration, "ckpt_dir": a.ckpt_dir}))
        return 0
    # held-out real windows: a fresh draw from the same panel with another seed
    hold = _dataset(s["data"], s["n_windows"], s["window"], s["features"], s["seed"] + 1000)
    fake = tr.generate(len(hold), seed=s["seed"] + 7)
    res = wasserstein_parity(tr.dataset.float().cpu().numpy(), hold, fake)
    res.update(model=a.model, preset=a.preset, iterations=tr.iteration, dtype=s["dtype"],
               batch_size=s["batch_size"], world=tr.world, seed=s["seed"],
               device=torch.cuda.get_device_name() if tr.device.type == "cuda" else "cpu")
    if a.preset == "reference" and s["window"] == 48 and s["features"] == 35 and s["data"] == "cleaned":
        try:  # the reference's own trained generator under the same protocol (absent data: skipped)
            anc = reference_anchor(seed=s["seed"])
            res.update(w_reference_generator=anc["w_fake_vs_real"], reference_generator=anc["generator"],
                       w_abs_diff_vs_reference=abs(res["w_fake_vs_real"] - anc["w_fake_vs_real"]))
        except FileNotFoundError:
            pass
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
        if a.save_fake:
            np.save(os.path.splitext(a.out)[0] + "_fake.npy", fake)
    return 0


def cmd_clean(a) -> int:
    from .data.cleaning import build_all

    out = build_all(a.raw, a.out)
    print(json.dumps({k: list(v.shape) for k, v in out.items()} if isinstance(out, dict) else str(out)))
    return 0


def cmd_replicate(a) -> int:
    from .data.io import load_cleaned
    from .finance import analytics
    from .finance.replication import LinearCloneBenchmark

    c = load_cleaned()
    hfd, etf, rf = c["hfd"], c["factor_etf_data"], c["rf"]
    half = len(hfd) // 2
    res = {}
    if a.method in ("linear", "all"):
        b = LinearCloneBenchmark(window=a.window).fit(etf.iloc[half:], hfd.iloc[half:], rf.iloc[half:])
        post = b.post()
        # excess-return Sharpe, as the AE clones' data_analysis (autoencoder_v4.ipynb:774, rf[-144:])
        rf_al = rf.iloc[:, 0].reindex(post.index).to_numpy(np.float64)
        real = hfd.reindex(post.index)
        res["linear"] = {
            "window": a.window, "months": int(len(post)),
            "period": [str(post.index[0].date()), str(post.index[-1].date())],
            "sharpe_ex_ante": {k: analytics.annualized_sharpe_ratio(b.ante_[k], rf_al) for k in post.columns},
            "sharpe_ex_post": {k: analytics.annualized_sharpe_ratio(post[k], rf_al) for k in post.columns},
            # the notebook's convention for the real index (hfd_res table, autoencoder_v4.ipynb:1015)
            "sharpe_real": {k: analytics.annualized_sharpe_ratio(real[k], rf_al) for k in post.columns},
            "turnover": dict(zip(post.columns, map(float, b.turnover()))),
        }
    dev = _device(a.device) if a.device != "cpu" else "cpu"
    dt = _torch_dtype(a.dtype)
    if a.method in ("ae", "all"):
        from .finance.autoencoder_replication import AE

        x_tr, x_te = etf.iloc[:half], etf.iloc[half:]
        y_tr, y_te = hfd.iloc[:half], hfd.iloc[half:]
        ae = AE(x_tr.to_numpy(), y_tr.to_numpy(), x_te.to_numpy(), y_te, a.latent, device=dev, dtype=dt, seed=a.seed)
        ae.train(verbose=0, plot=False)
        ante = ae.ante(rf.iloc[half:], y_te, window=a.window)
        post = ae.post(etf)
        rf_ae = rf.iloc[:, 0].reindex(post.index).to_numpy(np.float64)
        res["ae"] = {"latent": a.latent, "device": str(dev), "dtype": a.dtype,
                     "IS_r2": float(ae.model_IS_r2()), "IS_RMSE": float(ae.model_IS_RMSE()),
                     "OOS_r2": float(np.mean(ae.model_OOS_r2())), "OOS_RMSE": float(np.mean(ae.model_OOS_RMSE())),
                     "sharpe_ex_ante": {k: analytics.annualized_sharpe_ratio(ante[k], rf_ae) for k in ante.columns},
                     "sharpe_ex_post": {k: analytics.annualized_sharpe_ratio(post[k], rf_ae) for k in post.columns},
                     "turnover": dict(zip(post.columns, map(float, ae.turnover(c.get("hfd_fullname", {k: k for k in
                                                                                   post.columns}))["Turnover"])))}
    if a.method == "ae-sweep" and a.freq == "daily":
        from .data.io import load_daily_etf
        from .finance.experiment import daily_factor_study

        lo, _, hi = a.latents.partition("-")
        latents = list(range(int(lo), int(hi or lo) + 1))
        daily, _ = load_daily_etf()
        t0 = time.perf_counter()
        st = daily_factor_study(daily, latents=latents, seeds=[a.seed], device=dev, dtype=dt)
        res["ae_sweep_daily"] = {"device": str(dev), "dtype": a.dtype, "seed": a.seed, "rows": int(len(daily)),
                                 "period": [str(daily.index[0].date()), str(daily.index[-1].date())],
                                 "elapsed_s": round(time.perf_counter() - t0, 3),
                                 "fit_s": round(float(st["fit_s"].iloc[0]), 3),
                                 "metrics": st.set_index("latent").drop(columns=["seed", "fit_s"]).to_dict(orient="index")}
    elif a.method == "ae-sweep":
        from .finance.experiment import generated_augmentation, latent_sweep

        lo, _, hi = a.latents.partition("-")
        latents = range(int(lo), int(hi or lo) + 1)
        xe = ye = None
        if a.augment:
            xe, ye = generated_augmentation(np.load(a.augment, allow_pickle=False), c)
        t0 = time.perf_counter()
        sw = latent_sweep(c, latents=latents, window=a.window, x_extra=xe, y_extra=ye, verbose=True, device=dev,
                          dtype=dt, seed=a.seed)
        res["ae_sweep"] = {"device": str(dev), "dtype": a.dtype, "seed": a.seed, "augmented": bool(a.augment),
                           "elapsed_s": round(time.perf_counter() - t0, 3),
                           "metrics": sw.metrics.to_dict(orient="index"),
                           "sharpe_ante": sw.sharpe_ante.to_dict(orient="index"),
                           "turnover": sw.turnover.to_dict(orient="index"),
                           "sharpe_post": sw.sharpe_post.to_dict(orient="index"),
                           "best": sw.best.to_dict(orient="index")}
    print(json.dumps(res, indent=1, default=float))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1, default=float)
    return 0


def _torch_dtype(name: str):
    import torch

    return {"float32": torch.float32, "bfloat16": torch.bfloat16, "float64": torch.float64}[name]


def cmd_bench(a, rest) -> int:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench

    sys.argv = ["bench.py"] + rest
    return bench.main() or 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "bench":
        return cmd_bench(None, argv[1:])
    ap = argparse.ArgumentParser(prog="hfrep", description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    _add_train_args(sub.add_parser("train", help="train a GAN family"))
    pp = _add_train_args(sub.add_parser("parity", help="train, generate and report W-dist vs real windows"))
    pp.add_argument("--out", default=None)
    pp.add_argument("--save-fake", action="store_true")
    g = sub.add_parser("generate", help="generator checkpoint -> windows .npy")
    g.add_argument("--ckpt", required=True)
    g.add_argument("--n", type=int, default=1000)
    g.add_argument("--window", type=int, default=None)
    g.add_argument("--batch", type=int, default=4096)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--dtype", default="float32")
    g.add_argument("--device", default=None)
    g.add_argument("--out", required=True)
    e = sub.add_parser("eval", help="GAN_eval metrics of real vs generated windows")
    e.add_argument("--real", required=True)
    e.add_argument("--fake", required=True)
    e.add_argument("--name", default="model")
    e.add_argument("--metrics", default=None, help="comma list (default: run_all)")
    e.add_argument("--out", default=None)
    c = sub.add_parser("clean", help="raw data -> cleaned_data CSVs")
    c.add_argument("--raw", required=True)
    c.add_argument("--out", required=True)
    r = sub.add_parser("replicate", help="hedge-fund clone benchmarks")
    r.add_argument("--method", default="all", choices=["linear", "ae", "all", "ae-sweep"])
    r.add_argument("--latents", default="1-21", help="ae-sweep latent sizes, e.g. 1-21")
    r.add_argument("--freq", default="monthly", choices=["monthly", "daily"],
                   help="ae-sweep panel: the 337-month cleaned panel (reference) or the daily ETF excess-return "
                        "matrix (BASELINE config 2, data.cleaning.build_factor_etf_daily)")
    r.add_argument("--augment", default=None, help="ae-sweep: generated windows .npy (F=36) to add to training")
    r.add_argument("--window", type=int, default=24)
    r.add_argument("--latent", type=int, default=12)
    r.add_argument("--device", default="cpu", help="cpu | cuda (the autoencoder's training / inference device)")
    r.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "float64"])
    r.add_argument("--seed", type=int, default=123)
    r.add_argument("--out", default=None, help="also write the JSON result here")
    sub.add_parser("bench", help="flagship throughput benchmark (bench.py flags)")
    a = ap.parse_args(argv)
    return {"train": cmd_train, "parity": cmd_parity, "generate": cmd_generate, "eval": cmd_eval,
            "clean": cmd_clean, "replicate": cmd_replicate}[a.cmd](a)
