"""Wait states between an MFMA and the first instruction that reads its result, by consumer kind.

Straight-line scan (inside one basic block) of gfx950 assembly (hipcc -S): for every MFMA, walk
forward counting wait states (1 per instruction, N + 1 per `s_nop N`) to the first non-MFMA
instruction reading one of the MFMA's destination registers, and tabulate the gap per (MFMA opcode,
consumer class): plain VALU, PACKED fp32 VALU (v_pk_add/mul/fma_f32, which read a register pair), or
memory / accvgpr.  scripts/probes/mfma_pk_probe.hip measures on the hardware how many wait states
each consumer class needs; this lists what the compiler gives each class in the shipped kernels.

usage: python scripts/isa_pk_consumers.py FILE.s [FILE.s ...] [--show-below N]
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


def parse(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith(".") or s.endswith(":"):
        return None
    parts = s.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def classify(op):
    if op.startswith("v_pk_") and op.endswith("_f32"):
        return "pk_f32"
    if op.startswith(("buffer_store", "global_store", "ds_write", "flat_store", "scratch_store")):
        return "store"
    if op.startswith("v_accvgpr_read"):
        return "accvgpr_read"
    if op.startswith("v_"):
        return "valu"
    return "other"


def scan(path, show_below, fn_filter):
    lines = open(path).read().split("\n")
    table = defaultdict(lambda: defaultdict(list))
    fn = None
    for i, line in enumerate(lines):
        if re.match(r"^_Z\S*:", line):
            fn = line[:-1]
        p = parse(line)
        if not p or not p[0].startswith("v_mfma"):
            continue
        if fn_filter and (fn is None or fn_filter not in fn):
            continue
        op, ops = p
        dst = regs(ops[0]) if ops else set()
        ws = 0
        for j in range(i + 1, min(i + 200, len(lines))):
            l = lines[j]
            if re.match(r"^\.LBB|^_Z|^\s*s_(cbranch|branch|setpc|endpgm)", l.strip() if l.strip().startswith("s_") else l):
                break
            q = parse(l)
            if not q:
                continue
            qop, qops = q
            if qop == "s_nop":
                ws += int(qops[0], 0) + 1
                continue
            if qop.startswith("v_mfma"):
                ws += 1  # (an MFMA reading the result as SrcC is the chained case: not counted here)
                if dst & regs(",".join(qops[1:])):
                    break
                continue
            src = regs(",".join(qops[1:])) if not qop.startswith(("buffer_store", "global_store", "ds_write")) else regs(",".join(qops))
            if dst & src:
                cls = classify(qop)
                table[op][cls].append(ws)
                if show_below is not None and ws < show_below:
                    print(f"{path}:{j + 1}: {cls} {qop} {ws} wait states after {op} (line {i + 1}) in {fn[:70] if fn else '?'}")
                break
            ws += 1
            if dst & regs(qops[0] if qops else ""):
                break  # overwritten before read
    return table


def main(argv):
    show = None
    fn_filter = None
    files = []
    it = iter(argv)
    for a in it:
        if a == "--show-below":
            show = int(next(it))
        elif a == "--fn":
            fn_filter = next(it)
        else:
            files.append(a)
    total = defaultdict(lambda: defaultdict(list))
    for f in files:
        for op, d in scan(f, show, fn_filter).items():
            for cls, v in d.items():
                total[op][cls] += v
    for op in sorted(total):
        for cls in sorted(total[op]):
            v = total[op][cls]
            print(f"{op:28s} {cls:13s} n={len(v):6d} min={min(v):3d} max={max(v):3d}")


if __name__ == "__main__":
    main(sys.argv[1:])
