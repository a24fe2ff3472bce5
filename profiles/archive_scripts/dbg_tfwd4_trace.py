"""Fingerprint trace of the act = sigmoid bf16 tangent forward on lstm_fwd4<TAN> (variant built with
-DHFREP_TFWD4_SIGMOID=1 -DHFREP_FWD4_TRACE=1; profiles/r05_race): the tangent forward of one (x, v, primal
tape) runs N times, each into its own fingerprint buffer ([rb][t][wave][lane] x (tape xor, accumulator
registers 2 / 3 of the four gates, packed h tangent of rows 4 g + 2 / 3)).  For every run that differs
from the first: the first differing (step, row block, wave, lane) and which of the four words differ
there -- tape words (what the loads returned), accumulators (what the MFMAs produced) or only the
result (the cell math).   usage: python scripts/dbg_tfwd4_trace.py [B] [reps] [K]"""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
K = int(sys.argv[3]) if len(sys.argv) > 3 else 100
H, T, act, NCW = 100, 24, 1, 7
nrb = (B + 31) // 32
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
x, xd = mk(B, T, K), mk(B, T, K)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.randn(4 * H, device=dev, generator=g) * 0.1
hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
traces, outs = [], []
for r in range(reps):
    buf = torch.zeros(nrb, T, NCW, 64, 4, dtype=torch.int32, device=dev)
    ops.fwd4_trace(buf)
    hd, _ = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    torch.cuda.synchronize()
    ops.fwd4_trace(torch.empty(0, device=dev))
    traces.append(buf)
    outs.append(hd)
print(json.dumps({"B": B, "K": K, "reps": reps, "trace_written": int((traces[0] != 0).any(-1).sum().item())}), flush=True)
names = ["tape_xor", "acc_r2", "acc_r3", "h_tangent"]
for r in range(1, reps):
    nd_out = int((outs[0].view(torch.int16) != outs[r].view(torch.int16)).sum().item())
    d = traces[0] != traces[r]                      # [rb, t, wave, lane, 4]
    anyd = d.any(-1)
    rec = {"rep": r, "hd_ndiff": nd_out, "trace_entries_differing": int(anyd.sum().item())}
    if anyd.any():
        idx = anyd.nonzero()                        # rows: rb, t, wave, lane
        # first differing step per row block, then the earliest events
        tmin = idx[:, 1].min().item()
        first = idx[idx[:, 1] == tmin][:8]
        ev = []
        for rb, t, w, ln in first.tolist():
            ev.append({"rb": rb, "t": t, "wave": w, "lane": ln,
                       "differ": [names[i] for i in range(4) if bool(d[rb, t, w, ln, i])],
                       "run0": [hex(v & 0xffffffff) for v in traces[0][rb, t, w, ln].tolist()],
                       "runr": [hex(v & 0xffffffff) for v in traces[r][rb, t, w, ln].tolist()]})
        # per row block: the first step and which words differ at that step
        per = []
        for rb in sorted(set(idx[:, 0].tolist()))[:12]:
            sel = idx[idx[:, 0] == rb]
            t0 = sel[:, 1].min().item()
            s0 = sel[sel[:, 1] == t0]
            kinds = sorted({names[i] for rb_, t_, w_, l_ in s0.tolist() for i in range(4) if bool(d[rb_, t_, w_, l_, i])})
            per.append({"rb": rb, "first_t": t0, "waves": sorted(set(s0[:, 2].tolist())),
                        "lanes": sorted(set(s0[:, 3].tolist()))[:16], "differ": kinds})
        rec["first_events"] = ev
        rec["per_block_first_step"] = per
    print(json.dumps(rec), flush=True)
