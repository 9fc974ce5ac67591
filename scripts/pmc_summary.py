"""Summarise rocprofv3 --pmc counter CSVs for one kernel name substring (last dispatch)."""
import csv
import sys

sub = sys.argv[1]
for path in sys.argv[2:]:
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    if not rows:
        print(path, "no rows")
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    agg = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    r0 = [r for r in rows if int(r["Dispatch_Id"]) == last][0]
    dur = (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) / 1e3
    print(f"{path}: {r0['Kernel_Name'][:90]} dispatch {last} {dur:.1f} us VGPR={r0['VGPR_Count']} "
          f"AGPR={r0['Accum_VGPR_Count']} LDS={r0['LDS_Block_Size']} scratch={r0['Scratch_Size']}")
    waves = agg.get("SQ_WAVES", 0) or None
    for k, v in sorted(agg.items()):
        extra = f"  per-wave {v / waves:.4g}" if waves else ""
        print(f"  {k:28s} {v:.4g}{extra}")
