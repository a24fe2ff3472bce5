"""Probe which h row the split weight gradient pairs with each dZ row: dZ one-hot (row m -> column m)
for m < 400, h[m, u] = m, so gU[u, m] must be m - 1 (0 at sequence starts)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda", 0)
H, N, K = 100, 400, 100
for B, T in [(256, 32), (128, 64)]:
    M = B * T
    m = torch.arange(M, device=dev, dtype=torch.float32)
    hs = m[:, None].expand(M, H).reshape(B, T, H).contiguous()
    x = torch.zeros(B, T, K, device=dev)
    dz = torch.zeros(M, N, device=dev)
    dz[torch.arange(N), torch.arange(N)] = 1.0
    dz = dz.reshape(B, T, N)
    for impl in (1, 2):
        gW, gU, gb = torch.zeros(K, N, device=dev), torch.zeros(H, N, device=dev), torch.zeros(N, device=dev)
        Fn.lstm_wgrad_(x, hs, dz, gW, gU, gb, impl=impl)
        got = gU[0].cpu()
        exp = torch.tensor([0.0 if j % T == 0 else j - 1.0 for j in range(N)])
        bad = torch.nonzero(got != exp).flatten().tolist()
        print(f"B={B} T={T} impl={impl}: {len(bad)} bad; " +
              ", ".join(f"m={j}: got {got[j].item():.0f} exp {exp[j].item():.0f}" for j in bad[:10]), flush=True)
