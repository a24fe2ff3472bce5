"""Tangent reverse with an in-kernel generated head adjoint: run-to-run and vs materialized (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
# usage: python scripts/dbg_tbwd_gen.py [K ...]   (default K = 100; the r01 failures were at K = 32 / 35)
H, T, act = 100, 24, 2
for K, B in [(k, b) for k in ([int(a) for a in sys.argv[1:]] or [100]) for b in (32, 64, 256)]:
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)
    x, xd = mk(B, T, K), mk(B, T, K)
    W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
    b = torch.randn(4 * H, device=dev, generator=g) * 0.1
    hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    hds, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    d = mk(B, 1)
    hw = torch.randn(T * H, 1, device=dev, generator=g) * 0.1
    oa = Fn.OuterAdjoint(d, hw, (B, T, H))
    m = oa.materialize()
    for WW in (None, W):
        r1 = Fn.lstm_layer_tbwd(oa, oa, tape, ttape, U, act, W=WW)
        r2 = Fn.lstm_layer_tbwd(oa, oa, tape, ttape, U, act, W=WW)
        rm = Fn.lstm_layer_tbwd(m, m, tape, ttape, U, act, W=WW)
        rm2 = Fn.lstm_layer_tbwd(m, m, tape, ttape, U, act, W=WW)
        out0 = [round((p.float() - q.float()).abs().max().item(), 5) for p, q in zip(rm, rm2)]
        names = ["dZ", "dZd", "dX", "dXd"]
        out = {}
        for n, p, q, r in zip(names, r1, r2, rm):
            diff = (p.float() - q.float()).abs()
            out[n] = (round(diff.max().item(), 5), int((diff > 0).sum().item()),
                      round((p.float() - r.float()).abs().max().item(), 5))
            if diff.max() > 0:
                idx = (diff > 0).nonzero()
                out[n + "_where"] = (sorted(set(idx[:, 0].tolist()))[:8], sorted(set(idx[:, 1].tolist()))[:8],
                                     sorted(set(idx[:, 2].tolist()))[:12])
        print(K, B, "DX" if WW is not None else "noDX", "mat run-to-run", out0, out, flush=True)
