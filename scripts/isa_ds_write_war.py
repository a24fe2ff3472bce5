"""LDS-write data WAR census of gfx950 assembly (hipcc -S output): every ds_write whose DATA register a
following instruction overwrites within N wait states (before an lgkmcnt(0) wait).  Written for the
act = sigmoid tangent-forward drift (profiles/r05_race: the hypothesis was refuted).
usage: python scripts/isa_ds_write_war.py FILE.s [N]"""
import os
import re
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_mfma_war import regs, written
def ops_of(t):
    q=t.split(None,1); return q[0], ([o.strip() for o in re.split(r",\s*(?![^\[]*\])", q[1])] if len(q)>1 else [])
path=sys.argv[1]; lim=int(sys.argv[2]) if len(sys.argv)>2 else 3
L=[l.split(';')[0].strip() for l in open(path)]
hits=[]
for i,t in enumerate(L):
    if not t.startswith('ds_write') and not t.startswith('ds_store'): continue
    op,ops=ops_of(t)
    data=set()
    for o in ops[1:]:
        if o.startswith('offset'): continue
        data|=regs(o)
    ws=0
    for j in range(i+1,min(i+12,len(L))):
        u=L[j]
        if not u or u.startswith('.'):
            if u.startswith('.LBB'): break
            continue
        uop,uops=ops_of(u)
        if uop=='s_nop': ws+=int(uops[0],0)+1; continue
        if uop.startswith('s_waitcnt') and 'lgkmcnt(0)' in u: break
        w=written(uop,uops)
        if w & data:
            if ws<lim: hits.append((ws,i+1,t,u))
            break
        ws+=1
print(path.split('/')[-1], 'ds_write data overwritten within', lim, 'wait states:', len(hits))
for h in hits[:12]: print('  ', h[0], h[1], h[2][:50], '->', h[3][:50])
