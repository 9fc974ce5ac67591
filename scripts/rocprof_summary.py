"""Summarise a rocprofv3 --kernel-trace --stats run of `bench.py --serial` per P-frame and
(optionally) the FETCH_SIZE/WRITE_SIZE PMC passes, for comparison with bench.py's roofline.

usage: python scripts/rocprof_summary.py <stats_csv> <n_pframes_total> [fetch_csv write_csv]
"""
import csv
import sys

CONV_PREFIXES = ("conv_x3_kernel", "conv_mfma_f32_kernel", "conv_mfma_pipe_kernel", "deconv2_mfma_f32_kernel",
                 "conv_smalln_f32_kernel")


def is_conv(name):
    return any(p in name for p in CONV_PREFIXES)


def main():
    stats, nframes = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    conv = sum(float(r["TotalDurationNs"]) for r in rows if is_conv(r["Name"]))
    calls = sum(int(r["Calls"]) for r in rows if is_conv(r["Name"]))
    print(f"all kernels: {tot / 1e6:.2f} ms total, {tot / 1e6 / nframes:.3f} ms per P-frame")
    print(f"conv family: {conv / 1e6:.2f} ms total over {calls} launches, {conv / 1e6 / nframes:.3f} ms per P-frame")
    print("top kernels (ms per P-frame):")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
        print(f"  {float(r['TotalDurationNs']) / 1e6 / nframes:8.3f}  n/frame={int(r['Calls']) / nframes:6.1f}  {r['Name'][:100]}")
    if len(sys.argv) > 4:
        for label, path, col in (("FETCH", sys.argv[3], "FETCH_SIZE"), ("WRITE", sys.argv[4], "WRITE_SIZE")):
            rr = list(csv.DictReader(open(path)))
            kb = sum(float(r["Counter_Value"]) for r in rr if r.get("Counter_Name") == col and is_conv(r["Kernel_Name"]))
            corr = 2.0 if label == "FETCH" else 1.0  # gfx950: FETCH_SIZE reads 1/2 of wide streaming reads
            print(f"conv {label}: {kb * corr * 1024 / nframes / 1e9:.3f} GB per P-frame (corrected x{corr:g})")


if __name__ == "__main__":
    main()
