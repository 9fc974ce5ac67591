"""r6: which tap load and which wave lanes the wrong warp pixels of a LOCATE=10 race probe dump
(scripts/pipeline_race_probe.py) come from. usage: python scripts/race10_analyse.py race10_*.json"""
import json, sys, numpy as np
st = 8192*256
for fn in sys.argv[1:]:
    r=json.load(open(fn)); print('==',fn, r['summary'])
    from collections import Counter
    tapc=Counter(); lanes=Counter(); js=Counter(); quarters=Counter()
    for fr in r['frames']:
        W=3840
        for p in fr['pixels']:
            taps=p['taps']; wrong=np.array(p['wrong'])
            best=None
            for j,t in enumerate(taps):
                if t['w']<1e-3: continue
                others=sum(tt['w']*np.array(tt['val']) for k,tt in enumerate(taps) if k!=j)
                v=(wrong-others)/t['w']
                if np.abs(v).max()<2e-3:
                    best=j if best is None else (best if np.abs(v).max()>0 else j)
            # which two-tap zero combos?
            if best is None:
                import itertools
                for m in itertools.product((0,1),repeat=len(taps)):
                    if not any(m): continue
                    v=sum(t['w']*(0 if mk else np.array(t['val'])) for t,mk in zip(taps,m))
                    if np.abs(v-wrong).max()<1e-4: best=('zero',m); break
            tapc[str(best)]+=1
            q=p['y']*W+p['x']; j=q//st; th=q%st
            lanes[th%64]+=1; js[j]+=1; quarters[(th%64)//16]+=1
    print(' taps whose zeroing explains:',dict(tapc))
    print(' pixel iteration j (0,1 first pair; odd = p2):',dict(js))
    print(' lane quarter:',dict(quarters))
    print(' lanes:',sorted(lanes.items()))
