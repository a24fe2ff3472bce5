"""Split vs exact fp32 weight gradient on masked inputs: which chunk / part goes wrong."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda", 0)
H, N = 100, 400
for (B, T, K) in [(267, 24, 100), (267, 24, 32), (50, 4, 100)]:
    M = B * T
    g = torch.Generator(device=dev).manual_seed(1)
    x, hs, dz = (torch.randn(B, T, K, device=dev, generator=g), torch.randn(B, T, H, device=dev, generator=g),
                 torch.randn(B, T, N, device=dev, generator=g))
    rows = torch.arange(M, device=dev).reshape(B, T)
    for name, xm, hm, dm in [("all", 1, 1, None), ("x only", 1, 0, None), ("h only", 0, 1, None),
                             ("chunk0", 1, 1, 0), ("chunk1", 1, 1, 1)]:
        d = dz.clone()
        if dm is not None:
            d *= (((rows // 32) % 2) == dm).float()[..., None]
        outs = []
        for impl in (1, 2):
            gW, gU, gb = torch.zeros(K, N, device=dev), torch.zeros(H, N, device=dev), torch.zeros(N, device=dev)
            Fn.lstm_wgrad_(x * xm, hs * hm, d, gW, gU, gb, impl=impl)
            outs.append((gW, gU, gb))
        e = [(a - b).abs().max().item() for a, b in zip(outs[0], outs[1])]
        bad_cols = torch.nonzero((outs[0][0] - outs[1][0]).abs().amax(0) > 1e-3).flatten()
        bad_rows = torch.nonzero((outs[0][1] - outs[1][1]).abs().amax(1) > 1e-3).flatten()
        print(f"B={B} T={T} K={K} {name:7s}: max|exact-split| gW {e[0]:.2e} gU {e[1]:.2e} gb {e[2]:.2e}; "
              f"gW bad cols {bad_cols[:6].tolist()}..{bad_cols.numel()}, gU bad rows {bad_rows[:8].tolist()}", flush=True)
