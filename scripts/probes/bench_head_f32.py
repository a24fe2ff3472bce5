"""fp32 critic-head adjoint: lstmf BPTT / tangent reverse with the adjoint generated in-kernel (HEAD)
vs materialised (skinny dgrad + the plain kernels), B = 262 144, T = 24, K = 100, ms per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfrep.ops import functional as Fn  # noqa: E402

cuda = torch.device("cuda:0")
B, T, H, K, act = 262144, 24, 100, 100, 2
g = torch.Generator(device=cuda).manual_seed(3)
x = torch.randn(B, T, K, device=cuda, generator=g) * 0.5
xd = torch.randn(B, T, K, device=cuda, generator=g) * 0.5
W = torch.randn(K, 4 * H, device=cuda, generator=g) * 0.1
b = torch.zeros(4 * H, device=cuda)
U = torch.randn(H, 4 * H, device=cuda, generator=g) * 0.1
d = torch.randn(B, 1, device=cuda, generator=g)
w = torch.randn(T * H, 1, device=cuda, generator=g)
_, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
_, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
oa = Fn.OuterAdjoint(d, w, (B, T, H))


def timed(f, n=6):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {
    "bwd_head": timed(lambda: Fn.lstm_layer_bwd(oa, tape, U, act)),
    "bwd_materialised": timed(lambda: Fn.lstm_layer_bwd(oa.materialize(), tape, U, act)),
    "tbwd_head": timed(lambda: Fn.lstm_layer_tbwd(None, oa, tape, ttape, U, act)),
    "tbwd_materialised": timed(lambda: Fn.lstm_layer_tbwd(None, oa.materialize(), tape, ttape, U, act)),
}
print(json.dumps({"lib": os.environ.get("HFREP_NATIVE_LIB", "shipped"), **{k: round(v, 3) for k, v in res.items()}}))
