"""Scan gfx950 assembly (hipcc -S) for MFMA results read across a branch too early.

LLVM's hazard recognizer pads the wait states between an MFMA and a non-MFMA instruction that reads its
result (VALU, LDS / buffer store data, v_accvgpr_read) inside one basic block, but has missed the
case where the read sits behind a wave-uniform branch (an `if (wave_uniform) { mfma ... }` followed by
a use after the join): r02 found 2 wait states where >= 7 were needed (lstm_f32.hip wgrad note).  A
too-early read returns a stale accumulator; the result then depends on timing (run-to-run drift).

For every MFMA this walks the control flow forward (fall-through and branch targets) counting wait
states (1 per instruction, N + 1 per `s_nop N`) until MIN_WS, and reports a non-MFMA reader of the
MFMA's destination registers reached through at least one branch with fewer wait states than the
smallest gap the compiler itself chose for that opcode in straight-line code anywhere in the scanned
files (its own requirement).

usage: python scripts/isa_mfma_hazard.py FILE.s [FILE.s ...]   (exit 1 if any hazard is found)
"""
import re
import sys
from collections import defaultdict

MEASURED = {"v_mfma_f32_16x16x16_bf16": 6, "v_mfma_f32_16x16x32_bf16": 7}
MIN_WS = 20  # no gfx950 MFMA needs more (16-pass XDL write -> VALU read: 19 wait states)


def regs(tok, kind):
    out = set()
    for m in re.finditer(rf"\b{kind}\[(\d+):(\d+)\]", tok):
        out |= {(kind, r) for r in range(int(m.group(1)), int(m.group(2)) + 1)}
    for m in re.finditer(rf"(?<![\w\[:]){kind}(\d+)\b", tok):
        out.add((kind, int(m.group(1))))
    return out


def allregs(tok):
    return regs(tok, "v") | regs(tok, "a")


def operands(ins):
    return [o.strip() for o in ins.split(None, 1)[1].split(",")] if " " in ins else []


def reads(ins):
    """Registers an instruction reads (a VALU / MFMA / load writes its first operand)."""
    op = ins.split()[0]
    ops = operands(ins)
    if not ops:
        return set()
    if op.startswith(("ds_write", "ds_store", "buffer_store", "global_store", "scratch_store", "flat_store")):
        return set().union(*(allregs(o) for o in ops))
    if op.startswith(("v_", "ds_", "buffer_load", "global_load", "scratch_load", "flat_load")):
        return set().union(*(allregs(o) for o in ops[1:]))
    return set().union(*(allregs(o) for o in ops))


def parse(path):
    """{kernel: (instructions, {label: index})}"""
    kerns, kern, ins, labels = {}, None, [], {}
    for raw in open(path):
        l = raw.split(";")[0].strip()
        m = re.match(r"^(_Z\S*):", l)
        if m:
            if kern:
                kerns[kern] = (ins, labels)
            kern, ins, labels = m.group(1), [], {}
            continue
        if kern is None or not l:
            continue
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if l.startswith(".") or l.endswith(":"):
            if l.startswith(".Lfunc_end"):
                kerns[kern] = (ins, labels)
                kern = None
            continue
        ins.append(l)
    if kern:
        kerns[kern] = (ins, labels)
    return kerns


def succ(ins, labels, i):
    op = ins[i].split()[0]
    if op == "s_endpgm":
        return []
    if op == "s_branch":
        t = labels.get(ins[i].split()[1])
        return [t] if t is not None else []
    if op.startswith("s_cbranch"):
        t = labels.get(ins[i].split()[1])
        return [i + 1] + ([t] if t is not None else [])
    return [i + 1] if i + 1 < len(ins) else []


def ws_of(l):
    m = re.match(r"s_nop\s+(\d+)", l)
    return int(m.group(1)) + 1 if m else 1


def scan_kernel(ins, labels):
    """[(mfma index, reader index, wait states, crossed_branch)] for every reader within MIN_WS."""
    out = []
    for i, l in enumerate(ins):
        if not l.startswith("v_mfma"):
            continue
        dst = frozenset(allregs(operands(l)[0]))
        seen = {}
        stack = [(j, 0, False, dst) for j in succ(ins, labels, i)]
        while stack:
            j, ws, br, live = stack.pop()
            if j is None or j >= len(ins) or ws >= MIN_WS or not live:
                continue
            if seen.get((j, br, live), MIN_WS + 1) <= ws:
                continue
            seen[(j, br, live)] = ws
            lj = ins[j]
            op = lj.split()[0]
            if not op.startswith("v_mfma") and reads(lj) & live:
                out.append((i, j, ws, br))
                continue
            if op.startswith("v_mfma") and allregs(operands(lj)[0]) & live:
                continue  # overwritten / accumulated by a later MFMA: that one's readers are checked on their own
            if op.startswith(("v_", "ds_read", "ds_load", "buffer_load", "global_load", "scratch_load")) and operands(lj):
                live = live - allregs(operands(lj)[0])  # registers rewritten on this path hold new values
            nxt = succ(ins, labels, j)
            brn = br or op.startswith(("s_branch", "s_cbranch"))
            stack += [(k, ws + ws_of(lj), brn, live) for k in nxt]
    return out


def scan(paths):
    """Cross-branch reads with fewer wait states than the compiler's own straight-line minimum for the
    MFMA opcode, taken over every kernel of every file (its per-opcode requirement)."""
    found, need = [], defaultdict(lambda: MIN_WS)
    for p in paths:
        for k, (ins, labels) in parse(p).items():
            for i, j, ws, br in scan_kernel(ins, labels):
                op = ins[i].split()[0]
                found.append((p, k, ins[i], ins[j], ws, br))
                if not br:
                    need[op] = min(need[op], ws)
    # the compiler's straight-line minimum can only drop to the hardware need when that opcode has
    # straight-line readers at its minimum somewhere; cap it by the measured need (probes/mfma_raw_probe.hip,
    # probes/mfma_pk_probe.hip: v_mov / packed-fp32 readers, first clean wait-state count)
    for op, m in MEASURED.items():
        need[op] = min(need[op], m)
    return [(p, k, a, b, ws, need[a.split()[0]]) for p, k, a, b, ws, br in found if br and ws < need[a.split()[0]]]


if __name__ == "__main__":
    hits = scan(sys.argv[1:])
    for p, k, a, b, ws, need in hits:
        print(f"{p}: {k[:90]}\n    {a}\n    -> {b}   ({ws} wait states across a branch, straight-line minimum {need})")
    print(f"{len(hits)} cross-branch MFMA read hazards")
    sys.exit(1 if hits else 0)
