"""Run-to-run comparison of the bf16 tangent forward (act = sigmoid / tanh x K = 32 / 100): the shipped
library (tanh on lstm_fwd4<TAN>, sigmoid on lstm_tfwd2) or a variant built with -DHFREP_TFWD4_SIGMOID=1
(sigmoid on lstm_fwd4<TAN>, profiles/r05_race).  usage: python scripts/dbg_tfwd4_diag.py [B] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import _native  # noqa: E402
from hfrep.ops import functional as Fn  # noqa: E402

ops = _native.native()
dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32772
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
H, T = 100, 24
for act in (1, 2):
    for K in (32, 100):
        g = torch.Generator(device=dev).manual_seed(0)
        mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
        x, xd = mk(B, T, K), mk(B, T, K)
        W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
        U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
        b = torch.randn(4 * H, device=dev, generator=g) * 0.1
        hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
        t0 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
        nd, nprev = [], []
        prev = t0
        for _ in range(reps):
            t1 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
            d = (t0[0].view(torch.int16) != t1[0].view(torch.int16))
            nd.append(int(d.sum().item()))
            nprev.append(int((prev[0].view(torch.int16) != t1[0].view(torch.int16)).sum().item()))
            prev = t1
            if nd[-1]:
                idx = d.nonzero()
                rows = sorted(set((idx[:, 0] % 32).tolist()))
                blocks = sorted(set((idx[:, 0] // 32).tolist()))[:8]
                print(json.dumps({"act": act, "K": K, "rows_mod32": rows, "blocks": blocks,
                                  "steps": sorted(set(idx[:, 1].tolist()))[:12]}), flush=True)
        torch.cuda.synchronize()
        print(json.dumps({"act": act, "K": K, "B": B, "hd_ndiff_per_rep": nd, "hd_ndiff_vs_previous_rep": nprev,
                          "lib": os.environ.get("HFREP_NATIVE_LIB", "default")}), flush=True)
