"""Census of the MFMA region of one kernel in a gfx950 assembly file: between the first and the
last v_mfma (the step loop of the recurrent kernels), count MFMAs, scratch ops, exec-masked
branches, vmcnt waits and barriers.  usage: python scripts/isa_loops.py FILE.s NAME_SUBSTRING"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l) and pat in l.split(":")[0])
end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
body = src[start:end]
mf = [i for i, l in enumerate(body) if "v_mfma" in l]
seg = body[mf[0]:mf[-1] + 1] if mf else []
cnt = lambda p: sum(1 for l in seg if re.search(p, l))
print(f"MFMA region lines {mf[0] if mf else '-'}-{mf[-1] if mf else '-'}: mfma {cnt('v_mfma')}, scratch {cnt('scratch_')}, "
      f"exec-br {cnt('s_cbranch_exec')}, vmcnt-waits {cnt('s_waitcnt vmcnt')}, barriers {cnt('s_barrier')}")
