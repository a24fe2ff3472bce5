"""Static MFMA-result hazard census of gfx950 assembly (hipcc -S output).

For every v_mfma in a kernel, follow every control-flow path from it (fall-through, taken
conditional branches, unconditional branches) for up to ``--horizon`` wait states and find, on
each path, the first instruction that touches one of its destination registers other than as the
exact SrcC of a dependent MFMA (forwarded by the hardware).  Prints the wait states (instructions
+ s_nop counts) between producer and consumer, grouped by consumer opcode, and lists the pairs
below ``--min`` (default: passes + 4 for the MFMA's shape).  Used to compare a run-to-run
nondeterministic instantiation against its deterministic twins.

usage: python scripts/isa_mfma_hazards.py FILE.s NAME_SUBSTRING [--min N] [--show K] [--horizon W]
"""
import argparse
import re
from collections import defaultdict

PASSES = {"16x16x32": 8, "16x16x16": 8, "32x32x16": 16, "32x32x8": 16, "16x16x4": 8, "32x32x2": 16,
          "16x16x8": 8, "32x32x4": 16}


def regs(tok):
    """'v[4:7]' / 'a12' / 'v3' -> set of ('v'|'a', idx)."""
    out = set()
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]", tok):
        out |= {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    for m in re.finditer(r"(?<![\w\[:])([va])(\d+)\b", tok):
        out.add((m.group(1), int(m.group(2))))
    return out


def split_ops(code):
    parts = code.split(None, 1)
    if len(parts) < 2:
        return code, []
    return parts[0], [o.strip() for o in re.split(r",\s*(?![^\[]*\])", parts[1])]


def load(asm, name):
    src = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l) and name in l.split(":")[0])
    end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
    code, labels = [], {}  # (op, ops, text) per instruction; label -> index of the next instruction
    for l in src[start + 1:end]:
        c = l.split(";")[0].strip()
        if not c:
            continue
        if c.endswith(":"):
            labels[c[:-1]] = len(code)
            continue
        if c.startswith("."):
            continue
        op, ops = split_ops(c)
        code.append((op, ops, c))
    return code, labels


def consumers(code, labels, i, horizon):
    """{consumer index: (min wait states, text)} over all paths from MFMA i."""
    dst = regs(code[i][1][0])
    best, stack, seen = {}, [(i + 1, 0)], set()
    while stack:
        j, ws = stack.pop()
        while j < len(code) and ws <= horizon:
            if (j, ws) in seen:
                break
            seen.add((j, ws))
            opj, opsj, tj = code[j]
            if opj == "s_nop":
                ws += int(opsj[0], 0) + 1
                j += 1
                continue
            if (opj.startswith("v_mfma") and len(opsj) > 3 and regs(opsj[3]) == dst
                    and not ((regs(opsj[1]) | regs(opsj[2])) & dst)):
                break  # exact SrcC of a dependent MFMA: forwarded
            touched = set()
            for o in opsj:
                touched |= regs(o)
            if touched & dst:
                if j not in best or ws < best[j][0]:
                    best[j] = (ws, tj)
                break
            if opj.startswith("s_cbranch"):
                if opsj and opsj[0] in labels:
                    stack.append((labels[opsj[0]], ws + 1))
            elif opj == "s_branch":
                j, ws = labels.get(opsj[0], len(code)), ws + 1
                continue
            elif opj in ("s_endpgm", "s_setpc_b64"):
                break
            ws += 1
            j += 1
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("name")
    ap.add_argument("--min", type=int, default=0)
    ap.add_argument("--show", type=int, default=12)
    ap.add_argument("--horizon", type=int, default=40)
    a = ap.parse_args()
    code, labels = load(a.asm, a.name)
    hist, bad = defaultdict(list), []
    for i, (op, ops, text) in enumerate(code):
        if not op.startswith("v_mfma"):
            continue
        shape = next((k for k in PASSES if k in op), None)
        need = a.min or (PASSES.get(shape, 8) + 4)
        for j, (ws, tj) in consumers(code, labels, i, a.horizon).items():
            hist[tj.split()[0]].append(ws)
            if ws < need:
                bad.append((ws, need, i, j, text, tj))
    print(f"{a.name}: {sum(len(v) for v in hist.values())} MFMA -> consumer pairs (all paths, horizon {a.horizon})")
    for k, v in sorted(hist.items(), key=lambda kv: min(kv[1])):
        print(f"  {k:34s} n={len(v):4d} min={min(v):3d} median={sorted(v)[len(v) // 2]:3d}")
    bad.sort()
    print(f"  below threshold: {len(bad)}")
    for ws, need, i, j, text, tj in bad[:a.show]:
        print(f"    ws={ws:2d} need={need:2d} insn {i}->{j}: {text}  ->  {tj}")


if __name__ == "__main__":
    main()


def war_census(code, labels, horizon=24):
    """MFMA source operands (A, B and a SrcC that is not the destination) overwritten soon after
    the MFMA by a non-MFMA instruction: {(opcode of writer, operand kind): [wait states]}."""
    out = defaultdict(list)
    for i, (op, ops, text) in enumerate(code):
        if not op.startswith("v_mfma") or len(ops) < 4:
            continue
        srcs = {"A": regs(ops[1]), "B": regs(ops[2]), "C": regs(ops[3]) - regs(ops[0])}
        j, ws = i + 1, 0
        while j < len(code) and ws <= horizon:
            opj, opsj, tj = code[j]
            if opj == "s_nop":
                ws += int(opsj[0], 0) + 1
                j += 1
                continue
            if opj.startswith(("s_branch", "s_cbranch", "s_endpgm")):
                break
            if opsj and not opj.startswith(("v_mfma", "buffer_store", "ds_write", "global_store", "s_")):
                w = regs(opsj[0])
                for kind, rs in srcs.items():
                    if rs and w & rs:
                        out[(opj, kind)].append((ws, i, j))
            ws += 1
            j += 1
    return out
