"""fp32 LSTM input gradient dZ W^T: csrc/lstm_f32.hip lstmf_dgrad_kernel vs torch.mm (hipBLASLt).

usage: python scripts/dgrad_fp32_bench.py [M ...]   (GPU only; one JSON line per (M, KO))
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hfrep  # noqa: E402,F401
from hfrep.ops import _native  # noqa: E402


def timeit(fn, reps=10):
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
    Ms = [int(a) for a in sys.argv[1:]] or [786432, 6291456]
    g = torch.Generator(device=dev).manual_seed(0)
    for M in Ms:
        dz = torch.randn(M, 400, device=dev, generator=g)
        for KO in (100, 32):
            W = torch.randn(KO, 400, device=dev, generator=g) * 0.1
            fl = 2.0 * M * 400 * KO
            t_n = timeit(lambda: ops.lstmf_dgrad(dz, W, 1))
            t_s = timeit(lambda: ops.lstmf_dgrad(dz, W, 2))
            t_4 = timeit(lambda: ops.lstmf_dgrad(dz, W, 3))
            t_t = timeit(lambda: torch.mm(dz, W.t()))
            diff = (ops.lstmf_dgrad(dz, W, 1) - torch.mm(dz, W.t())).abs().max().item()
            diff_s = (ops.lstmf_dgrad(dz, W, 2) - ops.lstmf_dgrad(dz, W, 1)).abs().max().item()
            diff_4 = (ops.lstmf_dgrad(dz, W, 3) - ops.lstmf_dgrad(dz, W, 1)).abs().max().item()
            print(json.dumps({"op": "lstmf_dgrad", "M": M, "KO": KO, "native_ms": round(t_n, 3),
                              "split_ms": round(t_s, 3), "split_lds_ms": round(t_4, 3), "hipblaslt_ms": round(t_t, 3),
                              "native_tf": round(fl / t_n / 1e9, 1), "split_tf": round(fl / t_s / 1e9, 1),
                              "hipblaslt_tf": round(fl / t_t / 1e9, 1), "split_GBs": round(M * 400 * 4 / t_s / 1e6, 0),
                              "maxdiff": diff, "split_vs_exact_maxdiff": diff_s, "split_lds_vs_exact_maxdiff": diff_4}),
                  flush=True)
        del dz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
