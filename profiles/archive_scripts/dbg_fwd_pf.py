"""Forward with tape (two-step x prefetch) vs without tape (one-step): h must be bitwise equal."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
H = 100
for (B, T, K, act) in [(16, 24, 32, 1), (16, 24, 100, 1), (16, 24, 32, 2), (32, 24, 100, 2), (48, 24, 32, 2), (70, 24, 35, 1), (512, 24, 100, 2), (33, 7, 100, 0), (64, 25, 32, 2)]:
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(B, T, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
    b = torch.randn(4 * H, device=dev, generator=g) * 0.1
    h1, _ = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    h0 = Fn.lstm_layer_fwd(x, W, b, U, act, False)
    h0 = h0[0] if isinstance(h0, tuple) else h0
    d = (h1.float() - h0.float()).abs()
    bad = (d > 0).nonzero()
    print(dict(B=B, T=T, K=K, act=act, equal=torch.equal(h1, h0), maxdiff=d.max().item(),
               steps=sorted(set(bad[:, 1].tolist()))[:30], rows=sorted(set(bad[:, 0].tolist()))[:20]), flush=True)
