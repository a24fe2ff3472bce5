"""What FP3 planes (producer-side three-term bf16 split, csrc/lstm_f32.hip) would buy the fp32 consumers.

Times the fp32 weight-gradient kernels (quad K = 100, pair K = 32) and the split input gradient
(dgrad_s4, KO = 100) with every combination of operands handed over as pre-split planes (fp3_split)
instead of fp32, at the bench shape (B = 262 144 windows x T = 24, and the tangent segment where the
step has one), and checks that every plane variant is BITWISE equal to the fp32 variant (the planes are
a lossless encoding of the operands the consumers would otherwise split themselves).

usage: python scripts/bench_fp3.py [--batch 262144] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import _native  # noqa: E402


def timed(fn, iters):
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
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--T", type=int, default=24)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops = _native.native()
    dev = torch.device("cuda:0")
    H, N, T = 100, 400, a.T
    g = torch.Generator(device=dev).manual_seed(7)

    def mk(*s):
        return torch.randn(*s, device=dev, generator=g) * 0.5

    # ---- conversion cost and exactness
    d = mk(a.batch, T, N)
    p = ops.fp3_split(d, True)
    back = ops.fp3_join(p, True)
    print(json.dumps({"check": "fp3_roundtrip", "exact": bool(torch.equal(back, d))}), flush=True)
    ms = timed(lambda: ops.fp3_split(d, True), a.iters)
    print(json.dumps({"op": "fp3_split_400", "M": a.batch * T, "ms": round(ms, 4),
                      "GBps": round(d.numel() * 10 / ms / 1e6, 1)}), flush=True)
    del d, p, back
    torch.cuda.empty_cache()

    # ---- weight gradients: (K, impl, rows, tangent) as the step calls them
    for K, impl, B, tangent in [(100, 3, a.batch, True), (32, 2, a.batch, True), (100, 3, 2 * a.batch, False),
                                (32, 2, 2 * a.batch, False)]:
        prim = [mk(B, T, K), mk(B, T, H), mk(B, T, N)]
        tan = [mk(B, T, K), mk(B, T, H), mk(B, T, N)] if tangent else None
        planes = [ops.fp3_split(prim[0], False), ops.fp3_split(prim[1], False), ops.fp3_split(prim[2], True)]
        tplanes = ([ops.fp3_split(tan[0], False), ops.fp3_split(tan[1], False), ops.fp3_split(tan[2], True)]
                   if tangent else None)
        gW = torch.zeros(K, N, device=dev)
        gU = torch.zeros(H, N, device=dev)
        gb = torch.zeros(N, device=dev)
        base = None
        t0 = None
        for pm in (0, 4, 6, 7):
            ops_ = [planes[i] if pm & (1 << i) else prim[i] for i in range(3)]
            tops = ([tplanes[i] if pm & (1 << i) else tan[i] for i in range(3)] if tangent else [None] * 3)

            def call():
                ops.lstmf_wgrad_p_(*ops_, gW, gU, gb, *tops, impl)

            ms = timed(call, a.iters)
            gW.zero_(); gU.zero_(); gb.zero_()
            call()
            out = torch.cat([gW.flatten(), gU.flatten(), gb]).clone()
            if base is None:
                base, t0 = out, ms
            print(json.dumps({"op": "wgrad", "K": K, "impl": impl, "M": B * T, "tangent": tangent, "pm": pm,
                              "ms": round(ms, 4), "speedup_vs_fp32": round(t0 / ms, 3),
                              "bitwise_equal_fp32": bool(torch.equal(out, base))}), flush=True)
        del prim, tan, planes, tplanes
        torch.cuda.empty_cache()

    # ---- input gradient dX = dZ W^T, KO = 100 (split s4) and 32
    for KO in (100, 32):
        dz = mk(a.batch * T, N)
        W = mk(KO, N)
        dzp = ops.fp3_split(dz, True)
        t_f = timed(lambda: ops.lstmf_dgrad(dz, W, 3), a.iters)
        t_p = timed(lambda: ops.lstmf_dgrad_p(dzp, W, 3), a.iters)
        same = bool(torch.equal(ops.lstmf_dgrad(dz, W, 3), ops.lstmf_dgrad_p(dzp, W, 3)))
        t_e = timed(lambda: ops.lstmf_dgrad(dz, W, 1), a.iters)
        print(json.dumps({"op": "dgrad_s4", "KO": KO, "M": a.batch * T, "ms_fp32": round(t_f, 4),
                          "ms_planes": round(t_p, 4), "ms_exact": round(t_e, 4), "bitwise_equal_fp32": same}),
              flush=True)
        del dz, dzp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
