"""Timeline of the last N kernels of a rocprofv3 --kernel-trace directory: start offset, duration and
the gap to the previous kernel end, per kernel, with its queue (stream) id."""
import csv
import glob
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
skip_tail = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if skip_tail:
    rows = rows[:-skip_tail]
rows = rows[-last:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:7.2f}  gap {(s - prev_end) / 1e3:7.2f}  q{q:>3}  {name}")
    prev_end = max(prev_end, e)
