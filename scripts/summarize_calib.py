"""Counters of scripts/pmc_calib.sh divided by the known bytes of each calibration kernel
-> profiles/<tag>_pmc_calibration.json (usage: summarize_calib.py DIR [TAG])."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
tag = sys.argv[2] if len(sys.argv) > 2 else "r02"
COLS = 30
known = {}   # (kernel, grid threads) -> (read bytes, write bytes)
for n in (65536 * 3, 11184640):
    b = n * COLS * 4
    known[("rd_dword", n)] = (b, 0)
    known[("wr_dword", n)] = (0, b)
    known[("rd_x4", b // 16)] = (b, 0)
    known[("wr_x4", b // 16)] = (0, b)
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].strip()
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        if (name, grid) in known:
            vals[(name, grid, r["Counter_Name"])].append(float(r["Counter_Value"]) * 1024.0)
out = {"tag": tag, "unit": "counter bytes (KiB x 1024) / known bytes", "kernels": []}
for (name, grid), (rd, wr) in sorted(known.items()):
    e = {"kernel": name, "threads": grid, "known_read_bytes": rd, "known_write_bytes": wr,
         "where": "Infinity-Cache resident" if max(rd, wr) < 256 * 2 ** 20 else "past the 256 MB MALL"}
    for c, kb in (("FETCH_SIZE", rd), ("WRITE_SIZE", wr)):
        v = vals.get((name, grid, c))
        if v and kb:
            e[c + "_ratio"] = sorted(v)[len(v) // 2] / kb
            e[c + "_launches"] = len(v)
    out["kernels"].append(e)
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = os.path.join(root, "profiles", f"{tag}_pmc_calibration.json")
json.dump(out, open(p, "w"), indent=1)
print(json.dumps(out, indent=1))
