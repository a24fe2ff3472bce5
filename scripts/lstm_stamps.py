"""Phase timers of lstm_fwd2 (diagnostic build): python scripts/lstm_stamps.py  (sets HFREP_LSTM_DBG=64)."""
import json
import os
import sys

os.environ["HFREP_LSTM_DBG"] = str(64 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hfrep  # noqa: E402,F401
from hfrep.ops import _native  # noqa: E402
from hfrep.ops import functional as Fn  # noqa: E402

dev = torch.device("cuda:0")
B, T, K, H = int(os.environ.get("B", 16384)), 24, 100, 100
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(B, T, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
W = torch.randn(K, 4 * H, device=dev, generator=g) * 0.1
U = torch.randn(H, 4 * H, device=dev, generator=g) * 0.1
b = torch.zeros(4 * H, device=dev)
for _ in range(3):
    Fn.lstm_layer_fwd(x, W, b, U, 2, True)
torch.cuda.synchronize()
st = _native.native().lstm2_stamps().double()
nw = min(4096, (B + 63) // 64 * 8)  # waves that ran (2 tiles x 4 waves per workgroup)
st = st[:nw]
st = st[st.sum(1) > 0]
names = ["x_load_issue", "h_store", "mfma_x", "mfma_h", "gates_tape", "x_store_lds", "barrier", "loop_top"]
tot = st.sum(1).mean().item()
print(json.dumps({"waves": int(st.shape[0]), "cycles_per_wave": tot,
                  "share": {n: round(st[:, i].mean().item() / tot, 4) for i, n in enumerate(names)}}))
