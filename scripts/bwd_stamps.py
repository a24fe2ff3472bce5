"""Phase timers of lstm_bwd3 (diagnostic build, HFREP_LSTM_DBG=128): python scripts/bwd_stamps.py"""
import json
import os
import sys

os.environ["HFREP_LSTM_DBG"] = "128"
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
dH = (torch.randn(B, T, H, device=dev, generator=g) * 0.5).to(torch.bfloat16)
_, tape = Fn.lstm_layer_fwd(x, W, b, U, 2, True)
for _ in range(3):
    Fn.lstm_layer_bwd(dH, tape, U, 2, W=W)
torch.cuda.synchronize()
st = _native.native().lstm2_stamps().double().reshape(-1, 8, 8)  # [workgroup][wave][phase]
nwg = min(512, torch.cuda.get_device_properties(0).multi_processor_count)
st = st[:nwg]
rec = st[:, :4, :4].reshape(-1, 4)
dat = st[:, 4:, 4:].reshape(-1, 4)
tr, td = rec.sum(1).mean().item(), dat.sum(1).mean().item()
print(json.dumps({"cycles_per_wave": {"recurrence": tr, "data": td},
                  "recurrence": {n: round(rec[:, i].mean().item() / tr, 4) for i, n in
                                 enumerate(["prefetch_issue", "mfma", "gates", "barrier"])},
                  "data": {n: round(dat[:, i].mean().item() / td, 4) for i, n in
                           enumerate(["dh_load_issue", "dz_store", "dx_mfma_store_dh_lds", "barrier"])}}))
