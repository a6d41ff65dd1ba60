"""Per-kernel duration distribution (median / p10 / p90 / max) over the last 1 200 dispatches of a
rocprofv3 kernel trace, and the end-to-next-start gaps.  usage: python scripts/kernel_trace_dist.py trace.csv"""
import csv, sys, statistics, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = collections.defaultdict(list)
for r in rows[-1200:]:
    name = r["Kernel_Name"]
    key = "retrim" if "retrim_kernel" in name else ("step_ov" if "step_ov" in name else ("step" if "step_kernel" in name else name[:30]))
    by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    v.sort()
    print(f"{k:12s} n={len(v):5d} median {statistics.median(v):7.2f}  p10 {v[len(v)//10]:7.2f}  p90 {v[9*len(v)//10]:7.2f}  max {v[-1]:7.2f} us")
# gaps: start-to-start period of consecutive kernels
st = [int(r["Start_Timestamp"]) for r in rows[-1200:]]
en = [int(r["End_Timestamp"]) for r in rows[-1200:]]
gaps = sorted((st[i+1] - en[i]) / 1e3 for i in range(len(st)-1))
print("gap end->next start median %.2f p90 %.2f" % (statistics.median(gaps), gaps[9*len(gaps)//10]))
