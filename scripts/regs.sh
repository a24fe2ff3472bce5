#!/bin/bash
# per-kernel VGPR / AGPR / spill table of one .hip file.  usage: scripts/regs.sh csrc/file.hip
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics -I$(dirname $f) -c $f -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | python3 -c "
import sys,re
cur=None
rows=[]
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur={'name':m.group(1)}; rows.append(cur); continue
    for k in ('VGPRs','AGPRs','VGPRs Spill','Occupancy \[waves/SIMD\]'):
        m=re.search(r'remark:\s+'+k+r': (\d+)',l)
        if m and cur is not None: cur[k.split(' [')[0]]=m.group(1)
for r in rows: print(r.get('VGPRs'),r.get('AGPRs'),'spill',r.get('VGPRs Spill'),'occ',r.get('Occupancy'), r['name'][:90])
"
rm -f /tmp/regs_$$.o
