"""fp32 GEMM shapes of the training step: hfrep native kernels vs torch (hipBLASLt).

Prints one JSON line per (op, shape, impl) with ms and TFLOP/s.  GPU only.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hfrep  # noqa: E402,F401
from hfrep.ops import _native  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ops = _native.native()
    dev = torch.device("cuda")
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 786432
    g = torch.Generator(device=dev).manual_seed(0)
    for K, N in ((32, 400), (100, 400), (100, 32)):
        x = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(K, N, device=dev, generator=g) * 0.1
        b = torch.randn(N, device=dev, generator=g)
        fl = 2.0 * M * K * N
        t_n = timeit(lambda: ops.linear(x, W, b, 0))
        t_t = timeit(lambda: torch.addmm(b, x, W))
        err = (ops.linear(x, W, b, 0) - torch.addmm(b, x, W)).abs().max().item()
        print(json.dumps({"op": "linear", "M": M, "K": K, "N": N, "native_ms": round(t_n, 3), "torch_ms": round(t_t, 3),
                          "native_tf": round(fl / t_n / 1e9, 1), "torch_tf": round(fl / t_t / 1e9, 1), "maxdiff": err}))
        dz = torch.randn(M, N, device=dev, generator=g)
        t_n = timeit(lambda: ops.linear_dgrad(dz, W))
        t_t = timeit(lambda: dz @ W.t())
        print(json.dumps({"op": "dgrad", "M": M, "K": K, "N": N, "native_ms": round(t_n, 3), "torch_ms": round(t_t, 3),
                          "native_tf": round(fl / t_n / 1e9, 1), "torch_tf": round(fl / t_t / 1e9, 1)}))
        gW = torch.zeros(K, N, device=dev)
        gb = torch.zeros(N, device=dev)
        t_n = timeit(lambda: ops.linear_wgrad_(x, dz, gW, gb, 0))
        t_t = timeit(lambda: (gW.addmm_(x.t(), dz), gb.add_(dz.sum(0))))
        print(json.dumps({"op": "wgrad", "M": M, "K": K, "N": N, "native_ms": round(t_n, 3), "torch_ms": round(t_t, 3),
                          "native_tf": round(fl / t_n / 1e9, 1), "torch_tf": round(fl / t_t / 1e9, 1)}))
        del x, dz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
