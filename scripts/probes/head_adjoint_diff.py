"""Where the fp32 in-kernel head adjoint (lstmf_bwds HEAD) and the materialised dH disagree."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hfrep.ops import _native
from hfrep.ops import functional as Fn

cuda = torch.device("cuda:0")
B, T, H, K, act = 70, 24, 100, 100, 2
g = torch.Generator().manual_seed(71)
x = torch.randn(B, T, K, generator=g) * 0.5
W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
b = torch.randn(4 * H, generator=g) * 0.1
U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
d1 = torch.randn(B, 1, generator=g)
w = torch.randn(T * H, 1, generator=g)
xg, Wg, bg, Ug, d1g, wg = (t_.to(cuda) for t_ in (x, W, b, U, d1, w))
o1 = Fn.OuterAdjoint(d1g, wg, (B, T, H))
m1 = o1.materialize()
ref = (d1.double() * w.double().reshape(1, -1)).reshape(B, T, H)
print("materialised dH == d*w (fp32 product):", torch.equal(m1.cpu(), (d1 * w.reshape(1, -1)).reshape(B, T, H)),
      "max |m1 - ref|", (m1.double().cpu() - ref).abs().max().item())
_native.native().set_lstmf_bwd_impl(3)
_, tape = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
a = Fn.lstm_layer_bwd(o1, tape, Ug, act)
c = Fn.lstm_layer_bwd(m1, tape, Ug, act)
d = (a - c).abs()
print("max diff", d.max().item(), "n diff", (d > 0).sum().item(), "nan a/c", a.isnan().sum().item(), c.isnan().sum().item())
idx = (d > 0).nonzero()
print("first diffs (row, t, col):", idx[:12].tolist())
if len(idx):
    print("rows with diffs", sorted(set(idx[:, 0].tolist()))[:40])
    print("steps with diffs", sorted(set(idx[:, 1].tolist())))
    print("cols with diffs", sorted(set((idx[:, 2] % 100).tolist()))[:50])
