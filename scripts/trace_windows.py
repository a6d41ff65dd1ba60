"""The headline kernel in a rocprofv3 --kernel-trace of bench.py: per timed window (the step launches
between two clock_stamp_kernel dispatches), the average kernel duration and the average period
(start to start), beside the average over every dispatch of the kernel (ageing and pre-roll
included).  usage: python scripts/trace_windows.py <kernel_trace.csv> [out.json]"""
import csv
import json
import re
import statistics
import sys

STEP = re.compile(r"step_kernel<\d+, false, true, false, false, true, false>")   # the headline variant
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
allk, wins, cur = [], [], None
for r in rows:
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "clock_stamp_kernel" in name:
        if cur is None:
            cur = []
        else:
            wins.append(cur)
            cur = None
    elif STEP.search(name):
        allk.append((s, e))
        if cur is not None:
            cur.append((s, e))
out = {"dispatches": len(allk), "avg_us_all": statistics.mean(e - s for s, e in allk) / 1e3, "windows": []}
for w in wins:
    if len(w) < 2:
        continue
    d = [e - s for s, e in w]
    per = [(w[i + 1][0] - w[i][0]) for i in range(len(w) - 1)]
    out["windows"].append({"launches": len(w), "avg_kernel_us": statistics.mean(d) / 1e3,
                           "avg_period_us": statistics.mean(per) / 1e3})
if out["windows"]:
    out["median_window_avg_kernel_us"] = statistics.median(x["avg_kernel_us"] for x in out["windows"])
    out["median_window_avg_period_us"] = statistics.median(x["avg_period_us"] for x in out["windows"])
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
