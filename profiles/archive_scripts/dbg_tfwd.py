"""Locate tangent-forward errors by (row, step, unit) for one shape (debug aid)."""
import sys

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: F401
from hfrep.ops import functional as Fn
from hfrep.ops import reference as R

B, T, K, act = (int(v) for v in sys.argv[1:5])
H = 100
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(20)
x = (torch.randn(B, T, K, generator=g) * 0.5).to(torch.bfloat16)
W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
b = torch.randn(4 * H, generator=g) * 0.1
U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
hs, tape = Fn.lstm_layer_fwd(x.to(dev), W.to(dev), b.to(dev), U.to(dev), act, True)
zx = x.double() @ W.double() + b.double()
rh, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
ef = (hs.double().cpu() - rh).abs()
print("fwd err", ef.max().item())
badf = (ef > 0.05).nonzero()
if badf.shape[0]:
    print("fwd bad rows", sorted(set(badf[:, 0].tolist()))[:40])
    print("fwd bad steps", sorted(set(badf[:, 1].tolist())))
    print("fwd bad units", sorted(set(badf[:, 2].tolist()))[:60])
xd = (torch.randn(B, T, K, generator=g) * 0.3).to(torch.bfloat16)
hds, ttape = Fn.lstm_layer_tfwd(xd.to(dev), W.to(dev), tape, U.to(dev), act)
th, tz, tc = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), act)
e = (hds.double().cpu() - th).abs()
print("tfwd err", e.max().item())
bad = (e > 0.05).nonzero()
print("bad count", bad.shape[0])
if bad.shape[0]:
    print("rows", sorted(set(bad[:, 0].tolist()))[:40])
    print("steps", sorted(set(bad[:, 1].tolist())))
    print("units", sorted(set(bad[:, 2].tolist()))[:40])
    print("per-step max err", [round(e[:, t].max().item(), 3) for t in range(T)])
