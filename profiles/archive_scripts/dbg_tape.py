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
nrb = (B + 31) // 32
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, 2, True)
tp = tape.view(nrb, T, 4, 5, 2, 64, 8).float()
lane = torch.arange(64, device=dev)
wv = torch.arange(4, device=dev)
u = wv[:, None] * 32 + (lane[None, :] & 31)
valid = (u < H)  # [4][64]
# rows of block rb: row = rb*32 + acc32_row(r, lane), r = half*8 + i
for s in range(5):
    v = tp[:, :, :, s]  # nrb,T,4,2,64,8
    m = valid[None, None, :, None, :, None].expand_as(v)
    vv = v[m]
    print(f"tape slot {s}: nan={int((~torch.isfinite(vv)).sum())} sum={vv.double().abs().sum().item():.6e} absmax={vv.abs().max().item():.4e}", flush=True)
# per row-block / t nan map
bad = (~torch.isfinite(tp)) & valid[None, None, :, None, None, :, None]
if bad.any():
    idx = bad.nonzero()
    print("bad rb", sorted(set(idx[:, 0].tolist()))[:20], "t", sorted(set(idx[:, 1].tolist()))[:30], "w", sorted(set(idx[:, 2].tolist())), "slot", sorted(set(idx[:, 3].tolist())), flush=True)
