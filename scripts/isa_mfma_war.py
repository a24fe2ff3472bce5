"""MFMA source-operand WAR census of gfx950 assembly (hipcc -S output).

An MFMA reads its SrcA / SrcB at issue, but its SrcC (the accumulator input, 4 VGPRs per lane for a
16x16 tile) is read by the matrix pipe while the op is in flight.  A VALU / LDS-read / VMEM-load that
OVERWRITES one of those SrcC registers a few instructions after the MFMA issued can land before the
pipe has read it: the MFMA then accumulates onto the new value for the lanes / registers read last.
Written as a candidate for the act = sigmoid bf16 tangent forward's run-to-run rows-30/31 drift; the
A/B refuted it there (profiles/r05_race/README.md: an s_nop 7 behind the tails keeps the drift, and the
clean tanh instantiation has the same 3-4 wait-state pairs).  Kept as a census tool.

For every MFMA this walks forward in straight-line code (stopping at labels and branches) and records
the wait states (1 per instruction, N + 1 per s_nop N) before the first non-MFMA instruction that
writes a register of its SrcC (and, separately, of SrcA / SrcB, which are read at issue and are only
listed for reference).  Pairs below --min (default 8: one 16x16 op's pass count) are listed.

usage: python scripts/isa_mfma_war.py FILE.s [FILE.s ...] [--min N] [--kernel SUBSTR]
       (exit 1 if a SrcC pair below --min is found)
"""
import argparse
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


# instructions whose first operand is NOT a written VGPR
NO_VDST = re.compile(r"^(s_|ds_write|ds_store|buffer_store|global_store|flat_store|scratch_store|v_cmp|v_cmpx|"
                     r"exp|ds_gws|buffer_atomic|global_atomic)")


def written(op, ops):
    if NO_VDST.match(op) or not ops:
        return set()
    if op.startswith("v_readfirstlane") or op.startswith("v_readlane"):
        return set()  # (SGPR destination)
    return regs(ops[0])


def scan(files, kernel=None, horizon=40):
    tab = defaultdict(list)  # (opcode, 'srcc'|'srcab') -> gaps
    rows = []
    for path in files:
        lines = open(path).read().split("\n")
        fn = None
        for i, line in enumerate(lines):
            if re.match(r"^_Z\S*:", line):
                fn = line.split(":")[0]
            if kernel and (fn is None or kernel not in fn):
                continue
            s = line.split(";")[0].strip()
            if not s.startswith("v_mfma"):
                continue
            op, rest = s.split(None, 1)
            ops = [o.strip() for o in re.split(r",\s*(?![^\[]*\])", rest)]
            if len(ops) < 4:
                continue
            srcc = regs(ops[3]) - regs(ops[0])  # (an in-place accumulator is rewritten by the op itself)
            srcab = regs(ops[1]) | regs(ops[2])
            ws = 0
            found_c = found_ab = False
            for j in range(i + 1, min(i + 400, len(lines))):
                t = lines[j].split(";")[0].strip()
                if not t or t.startswith("."):
                    if t.startswith(".LBB"):
                        break
                    continue
                if re.match(r"^s_(cbranch|branch|setpc|endpgm)", t):
                    break
                q = t.split(None, 1)
                qop = q[0]
                qops = [o.strip() for o in re.split(r",\s*(?![^\[]*\])", q[1])] if len(q) > 1 else []
                if qop == "s_nop":
                    ws += int(qops[0], 0) + 1
                    continue
                if ws >= horizon:
                    break
                if qop.startswith("v_mfma"):
                    ws += 1
                    continue  # (the matrix pipe runs its ops in order)
                w = written(qop, qops)
                if not found_c and w & srcc:
                    tab[(op, "srcc")].append(ws)
                    rows.append((ws, path, j + 1, fn, op, t))
                    found_c = True
                if not found_ab and w & srcab:
                    tab[(op, "srcab")].append(ws)
                    found_ab = True
                if found_c and found_ab:
                    break
                ws += 1
    return tab, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--min", type=int, default=8)
    ap.add_argument("--kernel", default=None)
    a = ap.parse_args()
    tab, rows = scan(a.files, a.kernel)
    for (op, kind), gaps in sorted(tab.items()):
        print(f"{op:32s} {kind:6s} n={len(gaps):5d} min={min(gaps):3d} below {a.min}: {sum(g < a.min for g in gaps)}")
    bad = sorted(r for r in rows if r[0] < a.min)
    for ws, path, ln, fn, op, t in bad[:60]:
        print(f"  SrcC overwritten after {ws} wait states: {path}:{ln} {fn[:70]}  {op} -> {t[:70]}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
