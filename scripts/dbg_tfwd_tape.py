"""Which half of the bf16 tangent pair is run-to-run different at B ~ 32k, act = sigmoid (profiles/r03_race):
the tangent forward's tape (compared raw, and through the tangent reverse) or the tangent reverse itself
(run twice on ONE tangent tape).  usage: python scripts/dbg_tfwd_tape.py [B] [K] [act] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32772
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
act = int(sys.argv[3]) if len(sys.argv) > 3 else 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
H, T = 100, 24
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)
x, xd, dH = mk(B, T, K), mk(B, T, K), mk(B, T, H)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.randn(4 * H, device=dev, generator=g) * 0.1
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
t0 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
z0 = Fn.lstm_layer_tbwd(dH, dH, tape, t0[1], U, act)
for r in range(reps):
    t1 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    tt_eq = torch.equal(t0[1].view(torch.int16), t1[1].view(torch.int16))
    nd = int((t0[1].view(torch.int16) != t1[1].view(torch.int16)).sum().item())
    where = (t0[1].view(torch.int16) != t1[1].view(torch.int16)).nonzero().flatten()[:8].tolist()
    z1 = Fn.lstm_layer_tbwd(dH, dH, tape, t0[1], U, act)   # same tangent tape: the reverse alone
    z2 = Fn.lstm_layer_tbwd(dH, dH, tape, t1[1], U, act)   # the second tangent tape
    rev = [int((a_ != b_).sum().item()) for a_, b_ in zip(z0, z1)]
    via = [int((a_ != b_).sum().item()) for a_, b_ in zip(z0, z2)]
    dh = (t0[0].float() - t1[0].float()).abs()
    ih = (dh > 0).nonzero()
    if ih.numel():
        from collections import Counter
        print(dict(hd_maxdiff=dh.max().item(), hd_ndiff=int(ih.shape[0]),
                   hd_row_mod32=Counter((ih[:, 0] % 32).tolist()).most_common(12),
                   hd_steps=Counter(ih[:, 1].tolist()).most_common(6), hd_units=Counter(ih[:, 2].tolist()).most_common(8),
                   hd_row_blocks=len(set((ih[:, 0] // 32).tolist()))), flush=True)
    d = (z0[0].float() - z1[0].float()).abs()
    idx = (d > 0).nonzero()
    if idx.numel():
        from collections import Counter
        rows = Counter((idx[:, 0] % 32).tolist()).most_common(8)
        steps = Counter(idx[:, 1].tolist()).most_common(6)
        gates = Counter((idx[:, 2] // 100).tolist()).most_common(4)
        units = Counter((idx[:, 2] % 100).tolist()).most_common(8)
        blocks = len(set((idx[:, 0] // 32).tolist()))
        print(dict(maxdiff=d.max().item(), rel=(d.max() / z0[0].float().abs().max()).item(), row_mod32=rows, steps=steps,
                   gates=gates, units=units, row_blocks=blocks, of_blocks=(B + 31) // 32), flush=True)
    print(dict(B=B, K=K, act=act, rep=r, hd_equal=torch.equal(t0[0], t1[0]), ttape_equal=tt_eq, ttape_ndiff=nd,
               ttape_first=where, tbwd_same_tape_ndiff=rev, tbwd_other_tape_ndiff=via, numel=t0[1].numel()), flush=True)
