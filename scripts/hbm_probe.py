"""HBM reference rates on this GPU: device-to-device copy and a streaming read (sum), 4 GB."""
import json

import torch

dev = torch.device("cuda:0")
n = 2 * 1024 ** 3  # bf16 elements = 4 GB
x = torch.empty(n, dtype=torch.bfloat16, device=dev).normal_()
y = torch.empty_like(x)


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


ms = t(lambda: y.copy_(x))
print(json.dumps({"op": "copy", "GB": 8.59, "ms": round(ms, 3), "TBps": round(2 * n * 2 / ms / 1e9, 2)}))
ms = t(lambda: x.sum(dtype=torch.float32))
print(json.dumps({"op": "sum(read)", "GB": 4.29, "ms": round(ms, 3), "TBps": round(n * 2 / ms / 1e9, 2)}))
ms = t(lambda: y.fill_(1.0))
print(json.dumps({"op": "fill(write)", "GB": 4.29, "ms": round(ms, 3), "TBps": round(n * 2 / ms / 1e9, 2)}))
