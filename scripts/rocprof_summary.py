"""Summarise a rocprofv3 --kernel-trace --stats run of `bench.py --serial` per P-frame and
(optionally) the FETCH_SIZE/WRITE_SIZE PMC passes over the same command, for comparison with
bench.py's roofline object (which times the split-precision conv kernels -- conv_x3_kernel and
conv_wino_kernel -- with HIP events on their stream).

usage: python scripts/rocprof_summary.py <stats_csv> --bench-json bench_serial.json
           [--fetch fetch_counter_collection.csv --write write_counter_collection.csv
            --json-out profiles/r1/x3_traffic.json --height 1080 --width 1920]
"""
import argparse
import csv
import json

CONV_PREFIXES = ("conv_x3_kernel", "conv_dx_kernel", "conv_wino_kernel", "conv_wr7_kernel", "conv_stem_kernel", "conv_mfma_f32_kernel",
                 "conv_mfma_pipe_kernel",
                 "deconv2_mfma_f32_kernel", "conv_smalln_f32_kernel")
X3 = "conv_x3_kernel"
WINO = "conv_wino_kernel"
SPLIT = (X3, "conv_dx_kernel", WINO, "conv_wr7_kernel", "conv_stem_kernel")  # the split-precision family bench.py's roofline covers


def is_conv(name):
    return any(p in name for p in CONV_PREFIXES)


def pmc_per_dispatch(path, counter, sub):
    """{dispatch_id: value in bytes} for kernels whose name contains `sub` (counter unit: KiB)."""
    out = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") == counter and sub in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            out[d] = out.get(d, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("nframes", type=int, nargs="?", default=None,
                    help="P-frames the trace covers (default: derived from --bench-json and the launch count)")
    ap.add_argument("--bench-json", help="the profiled command's bench JSON: per-kernel launches and P-frames "
                    "per serial pass, so the P-frame count is derived from the trace's own launch count")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--json-out")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--gops-per-gpu", type=int, default=16, help="the profiled bench's GOPs per step")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    nframes = a.nframes
    if a.bench_json:
        # the trace may hold several serial passes (warm-up + timed); the P-frames it
        # covers = (split-family launches in the trace / launches per pass) x P-frames per pass
        b = json.load(open(a.bench_json))
        per_pass = sum(v["launches"] for k, v in b["roofline"]["per_kernel"].items() if k in SPLIT)
        pf_pass = round(b["value"] * b["ms_per_step"] / 1000.0 / b["n_gpus"])  # one rank's P-frames per step
        traced = sum(int(r["Calls"]) for r in rows if any(x in r["Name"] for x in SPLIT))
        if traced % per_pass:
            raise SystemExit(f"trace holds {traced} split launches, not a multiple of {per_pass} per pass")
        derived = traced // per_pass * pf_pass
        print(f"P-frames traced: {traced} split-family launches / {per_pass} per pass = {traced // per_pass} "
              f"passes x {pf_pass} P-frames = {derived}")
        if nframes is not None and nframes != derived:
            print(f"  (the given count {nframes} disagrees with the trace; using {derived})")
        nframes = derived
    if nframes is None:
        raise SystemExit("give the P-frame count or --bench-json")
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    conv = sum(float(r["TotalDurationNs"]) for r in rows if is_conv(r["Name"]))
    calls = sum(int(r["Calls"]) for r in rows if is_conv(r["Name"]))
    print(f"all kernels: {tot / 1e6:.2f} ms total, {tot / 1e6 / nframes:.3f} ms per P-frame")
    print(f"conv family: {conv / 1e6:.2f} ms total over {calls} launches, {conv / 1e6 / nframes:.3f} ms per P-frame")
    per = {}
    for k in SPLIT + ("split",):
        keys = SPLIT if k == "split" else (k,)
        ns = sum(float(r["TotalDurationNs"]) for r in rows if any(x in r["Name"] for x in keys))
        n = sum(int(r["Calls"]) for r in rows if any(x in r["Name"] for x in keys))
        per[k] = (ns, n)
        if n:
            label = "split-precision family (" + " + ".join(SPLIT) + ")" if k == "split" else f"{k} (all instantiations)"
            print(f"{label}: {n} launches, avg {ns / n / 1e3:.2f} us, {ns / 1e6 / nframes:.3f} ms per P-frame")
    x3_ns, x3_calls = per["split"]
    print("top kernels (ms per P-frame):")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
        print(f"  {float(r['TotalDurationNs']) / 1e6 / nframes:8.3f}  n/frame={int(r['Calls']) / nframes:6.1f}  "
              f"{r['Name'][:100]}")
    if a.fetch and a.write:
        # gfx950: FETCH_SIZE tallies 128-B requests at 64 B -> x2 (MI355X_MICROARCH.md, HBM section);
        # WRITE_SIZE exact for 16-B-per-lane stores (the x3 epilogue stores float4)
        out = {"height": a.height, "width": a.width, "gops_per_gpu": a.gops_per_gpu,
               "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE x1"}
        fam_f, fam_w = {}, {}
        for k in SPLIT:
            f = pmc_per_dispatch(a.fetch, "FETCH_SIZE", k)
            w = pmc_per_dispatch(a.write, "WRITE_SIZE", k)
            fam_f.update(f)
            fam_w.update(w)
            if not f:
                continue
            fb = 2.0 * sum(f.values()) / len(f)
            wb = sum(w.values()) / max(1, len(w))
            print(f"{k}: {len(f)} dispatches with FETCH_SIZE, {len(w)} with WRITE_SIZE; per launch "
                  f"fetch {fb / 1e6:.3f} MB (x2 corrected), write {wb / 1e6:.3f} MB")
            ns, n = per[k]
            out[k] = {"launches": len(f), "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                      "hbm_bytes_per_launch": round(fb + wb),
                      "avg_launch_us_kernel_trace": round(ns / n / 1e3, 2) if n else None}
        fb = 2.0 * sum(fam_f.values()) / max(1, len(fam_f))
        wb = sum(fam_w.values()) / max(1, len(fam_w))
        fc = 2.0 * sum(v for k, v in pmc_per_dispatch(a.fetch, "FETCH_SIZE", "").items()) / 1e9
        print(f"all kernels FETCH (x2): {fc:.3f} GB")
        # top-level fields: the split-precision family (bench.py's roofline object)
        out.update({"kernel": " + ".join(SPLIT), "launches": len(fam_f), "fetch_bytes_per_launch": round(fb),
                    "write_bytes_per_launch": round(wb), "hbm_bytes_per_launch": round(fb + wb),
                    "avg_launch_us_kernel_trace": round(x3_ns / x3_calls / 1e3, 2) if x3_calls else None})
        if a.json_out:
            with open(a.json_out, "w") as fo:
                json.dump(out, fo, indent=1)
            print("wrote", a.json_out)


if __name__ == "__main__":
    main()
