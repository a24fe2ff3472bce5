"""fp32 LSTM ops at the bench's W-term row count (2 x 262,144 rows): full-batch launch vs four
row slices.  Rows are independent in fwd / bwd / tfwd / tbwd / dgrad, so the outputs must be
bitwise equal; the weight gradient must equal the slice sum to fp32 reduction noise."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
T, H, S, act = 24, 100, 4, 2
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
rn = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
sl = lambda t, i: t[i * (B // S):(i + 1) * (B // S)].contiguous()  # noqa: E731


def report(name, full, parts):
    d = (full - torch.cat(parts, 0)).abs().max().item()
    print(f"{name:10s} max|full - slices| = {d:.3e}  (max|full| {full.abs().max().item():.3e})", flush=True)


for K in (32, 100):
    W, b, U = rn(K, 4 * H) / K ** 0.5, rn(4 * H) * 0.1, rn(H, 4 * H) / H ** 0.5
    x, dH, xd, dHd = rn(B, T, K), rn(B, T, H), rn(B, T, K), rn(B, T, H)
    print(f"K = {K}, B = {B}", flush=True)
    hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    res = [Fn.lstm_layer_fwd(sl(x, i), W, b, U, act, True) for i in range(S)]
    report("fwd h", hs, [r[0] for r in res])
    dZ = Fn.lstm_layer_bwd(dH, tape, U, act)
    dZs = [Fn.lstm_layer_bwd(sl(dH, i), res[i][1], U, act) for i in range(S)]
    report("bwd dZ", dZ, dZs)
    report("dgrad", Fn.linear_dgrad(dZ, W), [Fn.linear_dgrad(z, W) for z in dZs])
    hds, tt = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    tres = [Fn.lstm_layer_tfwd(sl(xd, i), W, res[i][1], U, act) for i in range(S)]
    report("tfwd hd", hds, [r[0] for r in tres])
    z1, z2 = Fn.lstm_layer_tbwd(dH, dHd, tape, tt, U, act)
    tb = [Fn.lstm_layer_tbwd(sl(dH, i), sl(dHd, i), res[i][1], tres[i][1], U, act) for i in range(S)]
    report("tbwd dZ", z1, [r[0] for r in tb])
    report("tbwd dZd", z2, [r[1] for r in tb])
    del tt, tres, tb, z1, z2
    gW, gU, gb = torch.zeros(K, 4 * H, device=dev), torch.zeros(H, 4 * H, device=dev), torch.zeros(4 * H, device=dev)
    Fn.lstm_wgrad_(x, hs, dZ, gW, gU, gb)
    sW, sU, sb = torch.zeros_like(gW), torch.zeros_like(gU), torch.zeros_like(gb)
    for i in range(S):
        Fn.lstm_wgrad_(sl(x, i), res[i][0], dZs[i], sW, sU, sb)
    for n, a, c in (("gW", gW, sW), ("gU", gU, sU), ("gb", gb, sb)):
        print(f"wgrad {n}: rel {((a - c).norm() / c.norm()).item():.3e}", flush=True)
    del hs, tape, res, dZ, dZs, x, dH, xd, dHd, hds
    torch.cuda.empty_cache()
