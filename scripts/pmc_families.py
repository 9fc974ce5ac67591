"""r6: per-family PMC summary of the bench's serial pass: for each split-precision
conv family (conv_x3 / conv_dx / conv_wino / conv_wr7 / conv_stem) the dispatch count and mean
duration, MFMA / VALU / SALU / LDS instruction counts and their ratios per MFMA, the MFMA-busy
fraction of every SIMD, the f16 MFMA FLOP issued per second, and HBM bytes (FETCH_SIZE x2 +
WRITE_SIZE, gfx950 correction) per launch.

usage: python scripts/pmc_families.py DIR_WITH_PASSES [--bench-json bench_serial.json] [--out file]
  every DIR/*/run_counter_collection.csv is one rocprofv3 --pmc pass over the same command
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (both summed over the
family's dispatches; GRBM_GUI_ACTIVE is the sum over the 8 XCDs); FLOP per MFMA instruction:
v_mfma_f32_32x32x16_f16 (x3, dx, stem) 32,768, v_mfma_f32_16x16x32_f16 (wino, wr7) 16,384.
"""
import argparse
import csv
import glob
import json
import os

FAMILIES = {"conv_x3_kernel": 32768, "conv_dx_kernel": 32768, "conv_wino_kernel": 16384,
            "conv_wr7_kernel": 16384, "conv_stem_kernel": 32768}
SIMDS, XCDS = 1024, 8


def family(name):
    for f in FAMILIES:
        if f in name:
            return f
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bench-json")
    ap.add_argument("--out")
    a = ap.parse_args()
    counters = {}   # family -> counter -> sum
    disp = {}       # family -> {dispatch id: duration ns} (per pass: the pass's own dispatch ids)
    for path in sorted(glob.glob(os.path.join(a.dir, "*", "run_counter_collection.csv"))):
        pass_disp = {}
        for r in csv.DictReader(open(path)):
            f = family(r["Kernel_Name"])
            if f is None:
                continue
            c = counters.setdefault(f, {})
            v = float(r["Counter_Value"])
            if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                v *= 1024.0  # KiB
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + v
            pass_disp.setdefault(f, {})[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for f, d in pass_disp.items():
            disp.setdefault(f, d)  # durations from the first pass (p1, the SQ one)
    lines, out = [], {}
    hdr = (f"{'family':18s} {'launches':>8s} {'avg us':>9s} {'MFMA busy':>9s} {'TF/s f16':>9s} {'VALU/MFMA':>9s} "
           f"{'SALU/MFMA':>9s} {'LDS/MFMA':>8s} {'HBM GB/launch':>13s} {'clock GHz':>9s}")
    lines.append(hdr)
    tot_flop = tot_ns = 0.0
    for f in FAMILIES:
        if f not in counters:
            continue
        c, d = counters[f], disp[f]
        n = len(d)
        ns = float(sum(d.values()))
        mf = c.get("SQ_INSTS_MFMA", 0.0)
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm / XCDS * SIMDS) if grbm else float("nan")
        flop = mf * FAMILIES[f]
        tflops = flop / (ns * 1e-9) / 1e12 if ns else float("nan")
        clock = grbm / XCDS / ns if ns else float("nan")
        hbm = (2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) / max(1, n)
        tot_flop += flop
        tot_ns += ns
        row = dict(launches=n, avg_us=ns / n / 1e3, mfma_busy=busy, f16_tflops_issued=tflops,
                   valu_per_mfma=c.get("SQ_INSTS_VALU", 0.0) / mf if mf else None,
                   salu_per_mfma=c.get("SQ_INSTS_SALU", 0.0) / mf if mf else None,
                   lds_per_mfma=c.get("SQ_INSTS_LDS", 0.0) / mf if mf else None,
                   hbm_bytes_per_launch=hbm, clock_ghz=clock, counters=c)
        out[f] = row
        lines.append(f"{f:18s} {n:8d} {row['avg_us']:9.1f} {busy * 100:8.1f}% {tflops:9.1f} "
                     f"{row['valu_per_mfma'] or 0:9.2f} {row['salu_per_mfma'] or 0:9.2f} {row['lds_per_mfma'] or 0:8.2f} "
                     f"{hbm / 1e9:13.3f} {clock:9.2f}")
    fam_tf = tot_flop / (tot_ns * 1e-9) / 1e12 if tot_ns else float("nan")
    lines.append(f"split family: {tot_flop / 1e12:.1f} TFLOP of f16 MFMA issued in {tot_ns / 1e6:.1f} ms of dispatches = "
                 f"{fam_tf:.1f} TF/s issued = {fam_tf / 2500:.3f} of the 2.5 PF dense f16 peak")
    out["split_family"] = dict(tflop_issued=tot_flop / 1e12, ms=tot_ns / 1e6, tflops_issued=fam_tf, frac_issued=fam_tf / 2500)
    if a.bench_json:
        b = json.load(open(a.bench_json))["roofline"]
        lines.append(f"bench line of {os.path.basename(a.bench_json)} (HIP events): frac_issued {b.get('frac_issued')}, "
                     f"issued {b.get('issued_tflops')} TF/s; algorithmic frac {b['frac']} ({b['achieved']} TF/s)")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as fo:
            fo.write(txt + "\n")
        with open(os.path.splitext(a.out)[0] + ".json", "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
