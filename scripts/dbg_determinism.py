"""Bitwise run-to-run check of the LSTM layer ops (debug aid): each op twice on the same inputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
H = 100
# usage: python scripts/dbg_determinism.py [BATCH_SCALE [REPEATS]]   (row counts x BATCH_SCALE)
SCALE = int(sys.argv[1]) if len(sys.argv) > 1 else 1
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 1
shapes = [(256, 24, 32, 1), (256, 24, 100, 1), (512, 24, 32, 2), (512, 24, 100, 2), (70, 24, 35, 2), (64, 24, 32, 0)]
for (B, T, K, act) in [(B * SCALE + (B % 7 if SCALE > 1 else 0), T, K, a) for (B, T, K, a) in shapes for _ in range(REPS)]:
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)
    x, xd, dH = mk(B, T, K), mk(B, T, K), mk(B, T, H)
    W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
    b = torch.randn(4 * H, device=dev, generator=g) * 0.1
    res = {}
    h1 = Fn.lstm_layer_fwd(x, W, b, U, act, False)
    h2 = Fn.lstm_layer_fwd(x, W, b, U, act, False)
    res["fwd_notape"] = torch.equal(h1[0], h2[0])
    hs1, tape1 = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    hs2, tape2 = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    res["fwd_h"] = torch.equal(hs1, hs2)
    # tapes compared through their consumer (padded-unit slots are never written)
    res["fwd_tape"] = torch.equal(Fn.lstm_layer_bwd(dH, tape1, U, act), Fn.lstm_layer_bwd(dH, tape2, U, act))
    t1 = Fn.lstm_layer_tfwd(xd, W, tape1, U, act)
    t2 = Fn.lstm_layer_tfwd(xd, W, tape1, U, act)
    res["tfwd_h"] = torch.equal(t1[0], t2[0])
    z1 = Fn.lstm_layer_tbwd(dH, dH, tape1, t1[1], U, act)
    z2 = Fn.lstm_layer_tbwd(dH, dH, tape1, t2[1], U, act)
    res["tfwd_tape"] = all(torch.equal(a_, b_) for a_, b_ in zip(z1, z2))
    # head-adjoint (in-kernel generated dH) variants
    d = mk(B, 1)
    hw = (torch.randn(T * H, 1, device=dev, generator=g) * 0.1)
    oa = Fn.OuterAdjoint(d, hw, (B, T, H))
    a1 = Fn.lstm_layer_bwd(oa, tape1, U, act, W=W)
    a2 = Fn.lstm_layer_bwd(oa, tape1, U, act, W=W)
    res["bwd_gen"] = all(torch.equal(p_, q_) for p_, q_ in zip(a1, a2))
    res["bwd_gen_vs_mat"] = all(torch.equal(p_, q_) for p_, q_ in zip(a1, Fn.lstm_layer_bwd(oa.materialize(), tape1, U, act, W=W)))
    g1 = Fn.lstm_layer_tbwd(oa, oa, tape1, t1[1], U, act, W=W)
    g2 = Fn.lstm_layer_tbwd(oa, oa, tape1, t1[1], U, act, W=W)
    res["tbwd_gen"] = all(torch.equal(p_, q_) for p_, q_ in zip(g1, g2))
    g3 = Fn.lstm_layer_tbwd(None, oa, tape1, t1[1], U, act, W=W)
    g4 = Fn.lstm_layer_tbwd(None, oa, tape1, t1[1], U, act, W=W)
    res["tbwd_gen_nodh"] = all(torch.equal(p_, q_) for p_, q_ in zip(g3, g4))
    print(dict(B=B, K=K, act=act, **res), flush=True)
