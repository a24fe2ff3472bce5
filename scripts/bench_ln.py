"""LayerNorm forward per-call time at the bench shape (rows = 262 144 x 24, D = 100): the native fast
path of csrc/misc.hip (layernorm_fwd_x4_kernel) for both dtypes, with / without the saved xhat / rstd and
the fused LeakyReLU prologue.  One JSON line per case: ms and the effective TB/s of its bytes.

    python scripts/bench_ln.py [--rows 6291456] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144 * 24)
    ap.add_argument("--D", type=int, default=100)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    import hfrep  # noqa: F401
    from hfrep.ops import functional as Fn

    dev = torch.device("cuda", 0)
    g = torch.randn(a.D, device=dev)
    b = torch.randn(a.D, device=dev)
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(a.rows, a.D, device=dev).to(dt)
        for save in (False, True):
            for pre in (False, True):
                fn = (lambda: Fn.lrelu_layer_norm_fwd(x, g, b, 1e-3, 0.2, save)) if pre else \
                    (lambda: Fn.layer_norm_fwd(x, g, b, 1e-3, save))
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                nb = x.numel() * x.element_size() * (3 if save else 2) + (a.rows * 4 if save else 0)
                print(json.dumps({"dtype": str(dt).split(".")[-1], "save": save, "lrelu": pre, "rows": a.rows,
                                  "D": a.D, "ms": round(ms, 4), "TB_s": round(nb / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
