"""Microbenchmark of the fused LSTM weight-gradient kernels at the flagship shapes.

Prints one line per (kernel, shape): time per call and the effective HBM rate of the bytes the op
must read (X, H, dZ once per segment).  Usage: python scripts/bench_wgrad.py [--batch 16384]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--T", type=int, default=24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float32"])
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    # bf16: impl 2 = tile kernel (gemm2), 0 = LDS-DMA streaming (wgrad3); fp32: 1 = exact MFMA, 2 = bf16 split
    impls, names = (((2, 0), {2: "wgrad2", 0: "wgrad3"}) if dt == torch.bfloat16 else
                    ((1, 2, 3), {1: "f32_exact", 2: "f32_split", 3: "f32_split_quad"}))
    dev = torch.device("cuda:0")
    H, N = 100, 400
    for K, rows_mult, tangent in [(32, 2, False), (100, 2, False), (32, 1, True), (100, 1, True)]:
        B = a.batch * rows_mult
        mk = lambda *s: (torch.randn(*s, device=dev) * 0.5).to(dt)  # noqa: E731
        x, hs, dZ = mk(B, a.T, K), mk(B, a.T, H), mk(B, a.T, N)
        seg = (mk(B, a.T, K), mk(B, a.T, H), mk(B, a.T, N)) if tangent else (None, None, None)
        gW = torch.zeros(K, N, device=dev)
        gU = torch.zeros(H, N, device=dev)
        gb = torch.zeros(N, device=dev)
        nbytes = (x.numel() + hs.numel() + dZ.numel()) * x.element_size() * (2 if tangent else 1)
        res = {}
        for impl in impls:
            for _ in range(3):
                Fn.lstm_wgrad_(x, hs, dZ, gW, gU, gb, *seg, impl=impl)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                Fn.lstm_wgrad_(x, hs, dZ, gW, gU, gb, *seg, impl=impl)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            res[impl] = ms
            print(json.dumps({"kernel": names[impl], "K": K, "M": B * a.T, "tangent": tangent,
                              "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
        # agreement of the two kernels on the same inputs
        outs = []
        for impl in impls:
            gW.zero_(); gU.zero_(); gb.zero_()
            Fn.lstm_wgrad_(x, hs, dZ, gW, gU, gb, *seg, impl=impl)
            outs.append(torch.cat([gW.flatten(), gU.flatten(), gb]).clone())
        for o, impl in zip(outs[1:], impls[1:]):
            rel = ((outs[0] - o).abs().max() / outs[0].abs().max()).item()
            print(json.dumps({"K": K, "tangent": tangent, "impl": names[impl], "maxrel_vs_first": rel,
                              "speedup": round(res[impls[0]] / res[impl], 2)}), flush=True)


if __name__ == "__main__":
    main()
