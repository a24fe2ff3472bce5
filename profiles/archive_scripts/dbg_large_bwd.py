"""fp32 BPTT full-batch vs 4 row slices (and a rerun of the full batch) at growing B."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import functional as Fn  # noqa: E402

T, H, S, act, K = 24, 100, 4, 2, 32
dev = torch.device("cuda", 0)
for B in [int(a) for a in sys.argv[1:]]:
    g = torch.Generator(device=dev).manual_seed(5)
    rn = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    sl = lambda t, i: t[i * (B // S):(i + 1) * (B // S)].contiguous()  # noqa: E731
    W, b, U = rn(K, 4 * H) / K ** 0.5, rn(4 * H) * 0.1, rn(H, 4 * H) / H ** 0.5
    x, dH = rn(B, T, K), rn(B, T, H)
    hs, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    dZ = Fn.lstm_layer_bwd(dH, tape, U, act)
    dZ2 = Fn.lstm_layer_bwd(dH, tape, U, act)
    parts = []
    for i in range(S):
        _, tp = Fn.lstm_layer_fwd(sl(x, i), W, b, U, act, True)
        parts.append(Fn.lstm_layer_bwd(sl(dH, i), tp, U, act))
    ref = torch.cat(parts, 0)
    bad = (dZ - ref).abs().amax(dim=(1, 2))
    rows = torch.nonzero(bad > 0).flatten()
    for r in rows[:6].tolist():
        d = (dZ[r] - ref[r]).abs()
        ts = torch.nonzero(d.amax(1) > 0).flatten().tolist()
        cols = torch.nonzero(d.amax(0) > 0).flatten()
        print(f"  row {r} (mod 32 = {r % 32}): steps {ts}; {cols.numel()} cols, units {sorted(set((cols % 100).tolist()))[:12]}")
    print(f"B={B}: rerun max diff {(dZ - dZ2).abs().max().item():.3e}; vs slices max {bad.max().item():.3e}, "
          f"{rows.numel()} bad rows, first {rows[:8].tolist()}, last {rows[-4:].tolist()}", flush=True)
    del hs, tape, dZ, dZ2, parts, ref, x, dH
    torch.cuda.empty_cache()
