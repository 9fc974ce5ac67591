"""Where the time of the overlapped timed region goes (rocprofv3 kernel trace of `bench.py`).

The timed region is found as the second long busy stretch after model load (warmup GOP, gap
from the synchronize, timed GOPs, gap, serial roofline pass). For each instant it records which
kernel classes run and prints the share of: conv running (alone / with other convs / with
rANS), rANS-only, other-only, idle; and the conv kernel-time inflation vs the serial pass.

usage: python scripts/gop_timeline.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# busy stretches separated by idle gaps > 0.3 ms
st = []
cs, ce = iv[0][0], iv[0][1]
for s, e, _ in iv:
    if s > ce + 300_000:
        st.append((cs, ce))
        cs, ce = s, e
    ce = max(ce, e)
st.append((cs, ce))
big = [x for x in st if x[1] - x[0] > 100e6]
t0, t1 = big[1]  # [0] warmup GOP, [1] timed GOPs, [2] serial roofline pass
s0, s1 = big[2]


def cls(n):
    return "conv" if "conv_" in n else ("rans" if "k_rans" in n else "other")


ev = []
for s, e, n in iv:
    s, e = max(s, t0), min(e, t1)
    if e > s:
        ev += [(s, 1, cls(n)), (e, -1, cls(n))]
ev.sort()
cnt = {"conv": 0, "rans": 0, "other": 0}
acc, last = {}, t0
for t, d, c in ev:
    if cnt["conv"]:
        key = "conv" if cnt["conv"] == 1 else "conv x%d" % min(cnt["conv"], 3)
        key += "+rans" if cnt["rans"] else ""
    else:
        key = "rans-only" if cnt["rans"] and not cnt["other"] else ("other" if cnt["other"] else "idle")
    acc[key] = acc.get(key, 0) + (t - last)
    cnt[c] += d
    last = t
tot = t1 - t0
print(f"timed window {tot / 1e6:.1f} ms")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:14s} {v / 1e6:8.1f} ms {100 * v / tot:5.1f} %")
ct = sum(min(e, t1) - max(s, t0) for s, e, n in iv if "conv_" in n and e > t0 and s < t1)
cser = sum(e - s for s, e, n in iv if "conv_" in n and s >= s0 and e <= s1)
print(f"conv kernel time: timed window {ct / 1e6:.1f} ms; serial pass (1 GOP) {cser / 1e6:.1f} ms")
