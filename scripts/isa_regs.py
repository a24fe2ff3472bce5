"""VGPR count and scratch bytes per kernel from a gfx950 assembly file (hipcc -S --cuda-device-only).

usage: python scripts/isa_regs.py FILE.s [substring]
"""
import re
import subprocess
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
vg = dict(re.findall(r"\.set (\S+)\.num_vgpr, (\d+)", src))
sc = dict(re.findall(r"\.set (\S+)\.private_seg_size, (\d+)", src))
names = [n for n in vg if pat in n]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    print(f"vgpr={vg[n]:>3} scratch={sc.get(n, '?'):>4}  {d.split('(')[0]}")
