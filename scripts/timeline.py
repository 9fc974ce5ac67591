"""GPU busy fraction from a rocprofv3 kernel trace (union of kernel intervals over a window).

usage: python scripts/timeline.py <kernel_trace.csv> [t0_frac t1_frac]
Prints the busy fraction of the whole trace span and, per 10 % slice, so the timed GOP of a
bench run can be read off; also the largest idle gaps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
if len(sys.argv) > 3:
    span = t1 - t0
    t0, t1 = t0 + int(float(sys.argv[2]) * span), t0 + int(float(sys.argv[3]) * span)
busy, cur_s, cur_e, gaps = 0, None, None, []
for s, e, n in iv:
    s, e = max(s, t0), min(e, t1)
    if e <= s:
        continue
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
print(f"window {(t1 - t0) / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms = {100 * busy / (t1 - t0):.1f} %")
gaps.sort(reverse=True)
print(f"idle gaps: {len(gaps)}, total {sum(g[0] for g in gaps) / 1e6:.2f} ms; largest:")
for g, at, n in gaps[:10]:
    print(f"  {g / 1e3:8.1f} us before {n}")
