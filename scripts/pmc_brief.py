"""Per-wave averages of the step kernel's PMC counters from scripts/ab_pmc.sh passes (rocprofv3 csv).
usage: python scripts/pmc_brief.py gpurun_out cur r02 65536"""
import csv
import glob
import os
import sys

root, variants, n = sys.argv[1], sys.argv[2:-1], sys.argv[-1]
for v in variants:
    tot, disp = {}, {}
    for f in glob.glob(os.path.join(root, f"pmc_{v}_{n}", "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "step_kernel" not in row.get("Kernel_Name", ""):
                continue
            c = row["Counter_Name"]
            tot[c] = tot.get(c, 0.0) + float(row["Counter_Value"])
            disp.setdefault(c, set()).add(row.get("Dispatch_Id"))
    if not tot:
        print(v, "no counters found")
        continue
    waves = tot.get("SQ_WAVES", 0) / max(1, len(disp.get("SQ_WAVES", [1])))
    out = {}
    for c, val in sorted(tot.items()):
        per_launch = val / max(1, len(disp[c]))
        out[c] = per_launch / waves if (waves and c.startswith("SQ_") and c != "SQ_WAVES") else per_launch
    print(v, "waves/launch", round(waves), {k: round(x, 1) for k, x in out.items()})
