"""Details of the act = sigmoid tangent-forward drift on lstm_fwd4<TAN> (variants built with
-DHFREP_TFWD4_SIGMOID=1): for every differing (row, step) -- values of both runs, the first differing step
of each row, non-finite counts of outputs and primal tape, and whether the first difference is in the
tangent h or in the tangent tape.  usage: python scripts/dbg_tfwd4_detail.py [B] [K] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32772
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
H, T, act = 100, 24, 1
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
x, xd = mk(B, T, K), mk(B, T, K)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.randn(4 * H, device=dev, generator=g) * 0.1
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
print(json.dumps({"nonfinite_primal_h": int((~torch.isfinite(hs.float())).sum()),
                  "nonfinite_primal_tape": int((~torch.isfinite(tape.float())).sum())}), flush=True)
t0 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
for r in range(reps):
    t1 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    a0, a1 = t0[0].float(), t1[0].float()
    d = t0[0].view(torch.int16) != t1[0].view(torch.int16)
    rows = d.any(dim=2).any(dim=1).nonzero().flatten().tolist()
    out = {"rep": r, "ndiff": int(d.sum()), "rows": len(rows), "nonfinite_run0": int((~torch.isfinite(a0)).sum()),
           "nonfinite_run1": int((~torch.isfinite(a1)).sum()),
           "tape_ndiff": int((t0[1].view(torch.int16) != t1[1].view(torch.int16)).sum())}
    print(json.dumps(out), flush=True)
    for row in rows[:6]:
        dr = d[row]
        steps = dr.any(dim=1).nonzero().flatten().tolist()
        s0 = steps[0]
        # per differing step: how many units differ and which 16-unit groups (compute wave of the unit)
        per_step = {int(st): [int(dr[st].sum()), sorted(set((dr[st].nonzero().flatten() // 16).tolist()))]
                    for st in steps}
        print(json.dumps({"row": row, "per_step": per_step}), flush=True)
        units = dr[s0].nonzero().flatten().tolist()
        print(json.dumps({"row": row, "row_mod32": row % 32, "block": row // 32, "first_step": s0,
                          "units_at_first": units[:12], "n_units_at_first": len(units),
                          "run0": [round(v, 6) for v in a0[row, s0, units[:6]].tolist()],
                          "run1": [round(v, 6) for v in a1[row, s0, units[:6]].tolist()],
                          "xd_row_absmax": float(xd[row].float().abs().max()),
                          "primal_h_row_first": [round(v, 4) for v in hs[row, s0, units[:4]].float().tolist()]}),
              flush=True)
