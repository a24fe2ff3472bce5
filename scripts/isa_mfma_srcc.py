"""MFMA -> MFMA SrcC dependencies across DIFFERENT opcodes, and the wait states the compiler put between.

A dependent MFMA whose SrcC is exactly the previous MFMA's destination issues back to back when both
are the SAME opcode (the matrix pipe forwards the accumulator).  When the opcodes differ -- a 16-wide
tail step (v_mfma_f32_16x16x16_bf16) or an exact-fp32 step (v_mfma_f32_16x16x4_f32) chained onto a
v_mfma_f32_16x16x32_bf16 accumulator -- the reader needs the writer's result in the register file.
This lists every such pair in straight-line code (gfx950 assembly from hipcc -S) with its gap
(1 per instruction, N + 1 per s_nop N), so it can be checked against scripts/probes/mfma_srcc_probe.hip.

usage: python scripts/isa_mfma_srcc.py FILE.s [FILE.s ...]   (exit 1 if a pair is below the measured need)
"""
import re
import sys
from collections import defaultdict


def regs(tok):
    out = set()
    for kind in ("v", "a"):
        for m in re.finditer(rf"\b{kind}\[(\d+):(\d+)\]", tok):
            out |= {(kind, r) for r in range(int(m.group(1)), int(m.group(2)) + 1)}
        for m in re.finditer(rf"(?<![\w\[:]){kind}(\d+)\b", tok):
            out.add((kind, int(m.group(1))))
    return out


# measured need (scripts/probes/mfma_srcc_probe.hip): 5 wait states for 16x16x32 <-> 16x16x16 bf16; the
# bf16 <-> fp32 pairs read correctly at 1
NEED = {("v_mfma_f32_16x16x32_bf16", "v_mfma_f32_16x16x16_bf16"): 5,
        ("v_mfma_f32_16x16x16_bf16", "v_mfma_f32_16x16x32_bf16"): 5}


def scan(files):
    """(table {(writer, reader, overlap): [gaps]}, hits [(path, line, fn, writer, reader, gap, need)])."""
    tab = defaultdict(list)
    hits = []
    for path in files:
        lines = open(path).read().split("\n")
        fn = None
        for i, line in enumerate(lines):
            if re.match(r"^_Z\S*:", line):
                fn = line.split(":")[0]
            s = line.split(";")[0].strip()
            if not s.startswith("v_mfma"):
                continue
            op, rest = s.split(None, 1)
            ops = [o.strip() for o in rest.split(",")]
            dst = regs(ops[0])
            ws = 0
            for j in range(i + 1, min(i + 80, len(lines))):
                t = lines[j].split(";")[0].strip()
                if not t or t.startswith("."):
                    if t.startswith(".LBB"):
                        break
                    continue
                if re.match(r"^s_(cbranch|branch|setpc|endpgm)", t):
                    break
                q = t.split(None, 1)
                qop = q[0]
                qops = [o.strip() for o in q[1].split(",")] if len(q) > 1 else []
                if qop == "s_nop":
                    ws += int(qops[0], 0) + 1
                    continue
                if qop.startswith("v_mfma") and len(qops) >= 4:
                    if regs(qops[3]) & dst:
                        if qop != op:
                            full = regs(qops[3]) == dst
                            tab[(op, qop, "exact" if full else "partial")].append(ws)
                            need = NEED.get((op, qop), 0)
                            if ws < need:
                                hits.append((path, j + 1, fn, op, qop, ws, need))
                        break
                    if regs(qops[0]) & dst or regs(",".join(qops[1:3])) & dst:
                        break
                elif regs(",".join(qops)) & dst:
                    break  # read or overwritten by a non-MFMA first
                ws += 1
    return tab, hits


def scan_cfg(files, horizon=8):
    """The same hand-over reached through control flow (a loop back-edge, a wave-uniform branch), which
    scan() stops at: for every MFMA walk fall-through and branch targets (isa_mfma_hazard's parser) until
    `horizon` wait states and report a later MFMA of the other bf16 opcode that reads the writer's
    destination as ANY source below the measured need.  [(path, kernel, writer, reader, ws, crossed)]"""
    from isa_mfma_hazard import parse, succ, ws_of, operands, allregs

    hits = []
    for path in files:
        for kern, (ins, labels) in parse(path).items():
            for i, l in enumerate(ins):
                if not l.startswith("v_mfma"):
                    continue
                opw = l.split()[0]
                dst = frozenset(allregs(operands(l)[0]))
                stack = [(j, 0, False) for j in succ(ins, labels, i)]
                seen = {}
                while stack:
                    j, ws, br = stack.pop()
                    if j >= len(ins) or ws >= horizon or seen.get((j, br), horizon + 1) <= ws:
                        continue
                    seen[(j, br)] = ws
                    lj = ins[j]
                    op = lj.split()[0]
                    ops = operands(lj)
                    if op.startswith("v_mfma"):
                        if op != opw and allregs(",".join(ops[1:])) & dst and ws < NEED.get((opw, op), 0):
                            hits.append((path, kern, l, lj, ws, br))
                        if allregs(ops[0]) & dst:
                            continue
                    elif op.startswith(("v_", "ds_read", "ds_load", "buffer_load", "global_load")) and ops \
                            and allregs(ops[0]) & dst:
                        continue  # destination rewritten on this path
                    crossed = br or op.startswith(("s_branch", "s_cbranch"))
                    stack += [(q, ws + ws_of(lj), crossed) for q in succ(ins, labels, j)]
    return hits


def main(argv):
    tab, hits = scan(argv)
    for path, kern, a, b, ws, br in scan_cfg(argv):
        print(f"{path}: {kern[:80]}: {b} reads {a} after {ws} wait states (through a branch: {br})")
        hits.append((path, 0, kern, a, b, ws, 5))
    for k in sorted(tab):
        v = tab[k]
        print(f"{k[0]:28s} -> {k[1]:28s} {k[2]:7s} n={len(v):5d} min={min(v):3d} max={max(v):3d}")
    for path, line, fn, op, qop, ws, need in hits:
        print(f"{path}:{line}: {qop} reads SrcC {ws} wait states after {op} (needs {need}) in {(fn or '?')[:80]}")
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
