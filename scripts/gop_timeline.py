"""Where the time of one overlapped GOP goes (rocprofv3 kernel trace of `bench.py`): for each
instant of the window, which kernel classes are running. Prints the time with a conv running,
with only rANS / only other kernels running, and idle, plus the GOP's tail after the last
encoder-side conv.

usage: python scripts/gop_timeline.py <kernel_trace.csv> <t0_frac> <t1_frac>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
T0, T1 = iv[0][0], max(e for _, e, _ in iv)
t0 = T0 + int(float(sys.argv[2]) * (T1 - T0))
t1 = T0 + int(float(sys.argv[3]) * (T1 - T0))


def cls(n):
    if "conv_" in n:
        return "conv"
    if "k_rans" in n:
        return "rans"
    return "other"


ev = []
for s, e, n in iv:
    s, e = max(s, t0), min(e, t1)
    if e > s:
        ev.append((s, 1, cls(n)))
        ev.append((e, -1, cls(n)))
ev.sort()
cnt = {"conv": 0, "rans": 0, "other": 0}
acc = {}
last = t0
for t, d, c in ev:
    key = "conv" if cnt["conv"] else ("rans-only" if cnt["rans"] and not cnt["other"] else
                                      ("other" if cnt["other"] else "idle"))
    acc[key] = acc.get(key, 0) + (t - last)
    cnt[c] += d
    last = t
acc["idle"] = acc.get("idle", 0) + (t1 - last)
tot = t1 - t0
print(f"window {tot / 1e6:.1f} ms")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:10s} {v / 1e6:8.2f} ms  {100 * v / tot:5.1f} %")
