"""Scan gfx950 assembly (hipcc -S) for the buffer-store data hazard the compiler misses.

A MUBUF store of more than 8 bytes (dwordx3 / dwordx4) whose data VGPRs a VALU instruction
overwrites in the very next instruction needs one wait state.  LLVM's hazard model only inserts
it when the store's soffset is not a register, but on gfx950 the hazard is there with an SGPR
soffset too: the store then writes the NEW register value (measured: lstm2.hip tape slots r01,
lstm_f32.hip lstmf_bwdp_kernel dZ rows 14 / 15 of a 32-row block r02, a few rows per 10^5).

usage: python scripts/isa_store_hazard.py FILE.s [FILE.s ...]   (exit 1 if any hazard is found)
"""
import re
import sys


def vregs(tok):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", tok):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"(?<![\w\[:])v(\d+)\b", tok):
        out.add(int(m.group(1)))
    return out


def scan(path):
    hits, kern = [], "?"
    lines = [l.split(";")[0].strip() for l in open(path)]
    ins = []
    for l in lines:
        m = re.match(r"^(_Z\S*):", l)
        if m:
            kern = m.group(1)
        if not l or l.startswith(".") or l.endswith(":"):
            continue
        ins.append((kern, l))
    for i, (k, l) in enumerate(ins[:-1]):
        m = re.match(r"buffer_store_(dwordx3|dwordx4|b96|b128)\s+(\S+),\s*(\S+),\s*(\S+),\s*(\S+)", l)
        if not m or not re.match(r"s\d+$", m.group(5)):
            continue
        data = vregs(m.group(2))
        nk, nxt = ins[i + 1]
        op = nxt.split()[0]
        if op.startswith("v_") and not op.startswith("v_mfma") and nk == k:
            dst = nxt.split(None, 1)[1].split(",")[0] if " " in nxt else ""
            if vregs(dst) & data:
                hits.append((k, l, nxt))
    return hits


if __name__ == "__main__":
    bad = 0
    for p in sys.argv[1:]:
        for k, st, nx in scan(p):
            bad += 1
            print(f"{p}: {k[:80]}\n    {st}\n    {nx}")
    print(f"{bad} store-data hazards")
    sys.exit(1 if bad else 0)
