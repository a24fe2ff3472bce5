"""Toolchain probe: load the in-tree kernel library on a GPU and check one fused op."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hfrep
from hfrep.ops import _native
print("cuda", torch.cuda.is_available(), torch.cuda.get_device_name(0) if torch.cuda.is_available() else None)
ops = _native.native()
n = 139601
p = torch.randn(n, device="cuda"); g = torch.randn(n, device="cuda"); ms = torch.rand(n, device="cuda")
p0, ms0 = p.clone(), ms.clone()
ops.rmsprop_(p, g, ms, 5e-5, 0.9, 1e-7, 0.0, 1.0)
msr = 0.9 * ms0 + 0.1 * g * g
pr = p0 - 5e-5 * g / (msr.sqrt() + 1e-7)
print("rmsprop max err", (p - pr).abs().max().item(), (ms - msr).abs().max().item())
print(torch.cuda.get_device_properties(0))
