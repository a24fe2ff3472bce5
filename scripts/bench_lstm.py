"""Microbenchmark of the LSTM v2 recurrent kernels (fwd / tangent fwd / BPTT / tangent reverse).

Times each layer-level op at the flagship shape (H=100, T=24, bf16) and prints one JSON line per op.
Usage: python scripts/bench_lstm.py [--batch 16384] [--K 100] [--iters 10] [--only fwd,bwd,...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--T", type=int, default=24)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--act", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="fwd,tfwd,bwd,tbwd,bwd_dx,tbwd_dx,dgrad")
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float32"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, T, K, H = a.batch, a.T, a.K, 100
    g = torch.Generator(device=dev).manual_seed(0)
    dt = getattr(torch, a.dtype)
    mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(dt)
    x, xd = mk(B, T, K), mk(B, T, K)
    W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
    b = torch.zeros(4 * H, device=dev)
    dH, dHd = mk(B, T, H), mk(B, T, H)
    hs, tape = Fn.lstm_layer_fwd(x, W, b, U, a.act, True)
    hds, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, a.act)
    dZ_ = Fn.lstm_layer_bwd(dH, tape, U, a.act)
    gW, gU, gb = torch.zeros(K, 4 * H, device=dev), torch.zeros(H, 4 * H, device=dev), torch.zeros(4 * H, device=dev)
    ops = {
        "fwd": lambda: Fn.lstm_layer_fwd(x, W, b, U, a.act, True),
        "fwd_notape": lambda: Fn.lstm_layer_fwd(x, W, b, U, a.act, False),
        "tfwd": lambda: Fn.lstm_layer_tfwd(xd, W, tape, U, a.act),
        "bwd": lambda: Fn.lstm_layer_bwd(dH, tape, U, a.act),
        "tbwd": lambda: Fn.lstm_layer_tbwd(dH, dHd, tape, ttape, U, a.act),
        "bwd_dx": lambda: Fn.lstm_layer_bwd(dH, tape, U, a.act, W=W),
        "tbwd_dx": lambda: Fn.lstm_layer_tbwd(dH, dHd, tape, ttape, U, a.act, W=W),
        "dgrad": lambda: Fn.linear_dgrad(dZ_, W),
        "wgrad": lambda: Fn.lstm_wgrad_(x, hs, dZ_, gW, gU, gb),
        "wgrad_tan": lambda: Fn.lstm_wgrad_(x, hs, dZ_, gW, gU, gb, xd, hds, dZ_),
    }
    for name in a.only.split(","):
        ms = timeit(ops[name], a.iters)
        print(json.dumps({"op": name, "dtype": a.dtype, "B": B, "T": T, "K": K, "ms": round(ms, 4),
                          "us_per_step": round(ms * 1e3 / T, 2)}), flush=True)


if __name__ == "__main__":
    main()
