#!/bin/bash
# kernel resource usage table for one .hip file: name VGPR AGPR spill occupancy
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | sed -n 's/.*remark: \(.*\) \[-Rpass.*/\1/p' | python3 -c "
import sys,re,subprocess
rows=[];cur=None
for l in sys.stdin:
    l=l.strip()
    if l.startswith('Function Name:'):
        n=l.split(':',1)[1].strip()
        try: n=subprocess.run(['c++filt',n],capture_output=True,text=True).stdout.strip()
        except Exception: pass
        cur={'name':n};rows.append(cur)
    elif cur is not None and ':' in l:
        k,v=l.split(':',1);cur[k.strip()]=v.strip()
for r in rows:
    print(f\"{r.get('VGPRs','?'):>4} {r.get('AGPRs','?'):>4} spill={r.get('VGPRs Spill','?'):>5} occ={r.get('Occupancy [waves/SIMD]','?')} {r['name'][:110]}\")
"
