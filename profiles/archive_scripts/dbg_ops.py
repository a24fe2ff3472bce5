"""Debug: checksums of every LSTM v2 op output at a bench shape (compare two library builds)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hfrep  # noqa
from hfrep.ops import functional as Fn
dev = torch.device("cuda:0")
B, T, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
H = 100
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)
x, xd = mk(B, T, K), mk(B, T, K)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.zeros(4 * H, device=dev)
dH, dHd = mk(B, T, H), mk(B, T, H)
def cs(name, t):
    t = t.float()
    print(f"{name:8s} nan={int((~torch.isfinite(t)).sum())} sum={t.double().abs().sum().item():.6e}", flush=True)
def fill(t):
    return t
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, 2, True)
cs("hs", hs)
hs0, _ = Fn.lstm_layer_fwd(x, W, b, U, 2, False)
cs("hs_notape", hs0)
hds, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, 2)
cs("hds", hds)
torch.cuda.synchronize()
dZ = Fn.lstm_layer_bwd(dH, tape, U, 2); cs("dZ", dZ)
dZ1, dX = Fn.lstm_layer_bwd(dH, tape, U, 2, W=W); cs("dZ_dx", dZ1); cs("dX", dX)
dZn, dXn = Fn.lstm_layer_bwd(dH, tape, U, 2, W=W, need_dz=False); cs("dX_nodz", dXn)
a = Fn.lstm_layer_tbwd(None, dHd, tape, ttape, U, 2); cs("tz", a[0]); cs("tzd", a[1])
a = Fn.lstm_layer_tbwd(dH, dHd, tape, ttape, U, 2, W=W); cs("tz_dx", a[0]); cs("tzd_dx", a[1]); cs("tx", a[2]); cs("txd", a[3])
