"""Median duration (last 1000 launches) of each kernel in a rocprofv3 --kernel-trace directory."""
import csv
import glob
import statistics
import sys

d, label = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
by = {}
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(label)
for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= 50:
        print(f"   {n[:70]:70s} n={len(v):6d} median {statistics.median(v[-1000:]):8.2f} us")
