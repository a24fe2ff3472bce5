"""Hypothesis check for the act = sigmoid bf16 tangent-forward drift (variant -DHFREP_TFWD4_SIGMOID=1,
profiles/r05_race): the h tangent of row 30 (31) of a 32-row block is written to the LDS h tile by a
ds_write_b16 whose data register the next VALU instruction overwrites with the value of row 31 (the next
ds_write's data).  If the write reads its data late, row 30 gets row 31's value.  For every run that
differs from run 0: at each differing row's FIRST differing step, compare the differing units' values
with run 0's values of the partner row (30 <-> 31) at the same step.
usage: python scripts/dbg_tfwd4_rowswap.py [B] [reps] [K]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32772
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
K = int(sys.argv[3]) if len(sys.argv) > 3 else 100
H, T, act = 100, 24, 1
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
x, xd = mk(B, T, K), mk(B, T, K)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.randn(4 * H, device=dev, generator=g) * 0.1
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
h0 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)[0].view(torch.int16)
tot = {"cells": 0, "equal_partner_row": 0, "equal_partner_row_prev_step": 0}
for r in range(1, reps):
    h1 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)[0].view(torch.int16)
    d = h0 != h1                                   # (B, T, H)
    rows = d.any(-1).any(-1).nonzero().flatten().tolist()
    ev = []
    for row in rows:
        steps = d[row].any(-1).nonzero().flatten()
        t = int(steps.min())
        units = d[row, t].nonzero().flatten()
        pr = row + 1 if row % 32 == 30 else row - 1 if row % 32 == 31 else None
        if pr is None or pr >= B:
            ev.append({"row": row, "t": t, "row_mod32": row % 32, "n_units": len(units)})
            continue
        got = h1[row, t, units]
        partner = h0[pr, t, units]
        eq = int((got == partner).sum())
        eqp = int((got == h0[pr, t - 1, units]).sum()) if t > 0 else 0
        tot["cells"] += len(units)
        tot["equal_partner_row"] += eq
        tot["equal_partner_row_prev_step"] += eqp
        ev.append({"row": row, "row_mod32": row % 32, "t": t, "units": units.tolist()[:16], "n_units": len(units),
                   "equal_to_partner_row_same_step": eq, "equal_to_partner_row_prev_step": eqp})
    print(json.dumps({"rep": r, "rows_differing": len(rows), "first_step_events": ev[:12]}), flush=True)
print(json.dumps({"total": tot}), flush=True)
