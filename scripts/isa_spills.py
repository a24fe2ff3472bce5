"""Where a kernel's scratch spills / reloads sit relative to its loops (gfx950 assembly).

usage: python scripts/isa_spills.py FILE.s MANGLED_NAME_SUBSTRING
Prints the loop headers and the scratch instructions in order, with line numbers.
"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(src) if l.startswith("_Z") and pat in l and l.rstrip().endswith(":") is False or
             (l.startswith("_Z") and pat in l and ":" in l and not l.startswith("\t")))
end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
for i in range(start, end):
    l = src[i]
    if "Loop Header" in l or "scratch_" in l or re.search(r"s_cbranch_\w+ \.LBB", l):
        print(i - start, l.strip()[:90])
