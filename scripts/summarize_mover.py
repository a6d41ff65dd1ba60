"""Summarise scripts/r05_mover_prof.sh: per mover case, the traced average launch duration, the PMC
traffic per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB, the gfx950 correction of MI355X_MICROARCH.md)
and the achieved rate of the 315 bytes per env the step kernel moves.  Writes
profiles/r05_mover_4m_pmc_summary.json and copies the kernel stats of case 5."""
import csv
import glob
import json
import os
import shutil
import sys

d, n = sys.argv[1], int(sys.argv[2])   # d = "-": keep the committed PMC cases, update the period only
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
summary = os.path.join(root, "profiles", "r05_mover_4m_pmc_summary.json")
out = {"envs": n, "bytes_per_env": 315, "source": "scripts/ubench/mover.hip via scripts/r05_mover_prof.sh", "cases": {}}
if d == "-":
    out = json.load(open(summary))
for c, label in (("5", "12 waves per CU (the bulk step kernel's occupancy), no arithmetic"),
                 ("9", "12 waves per CU, 1 700 VALU per lane between the loads and the stores")):
    if d == "-":
        break
    durs = []
    for f in glob.glob(os.path.join(d, f"trace{c}", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "mover" in r["Kernel_Name"]:
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = {}
    for f in glob.glob(os.path.join(d, f"pmc{c}_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "mover" in r.get("Kernel_Name", ""):
                cnt.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in cnt.items()}
    e = {"label": label, "launches_traced": len(durs)}
    if durs:
        avg = sum(durs) / len(durs)
        e["kernel_avg_us_trace"] = avg / 1e3
        e["achieved_GBs_315"] = 315 * n / avg
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd, wr = 2 * mean["FETCH_SIZE"] * 1024, mean["WRITE_SIZE"] * 1024
        e.update(hbm_read_bytes_per_launch=rd, hbm_write_bytes_per_launch=wr, hbm_bytes_per_launch=rd + wr,
                 traffic_over_moved=(rd + wr) / (315 * n), moved_read=128 * n, moved_write=187 * n)
    out["cases"][c] = e
    stats = glob.glob(os.path.join(d, f"trace{c}", "**", "*kernel_stats.csv"), recursive=True)
    if stats and c == "5":
        shutil.copy(stats[0], os.path.join(root, "profiles", "r05_mover_4m_kernel_stats.csv"))
# the event-timed sweeps of the same binary (100 launches per hipGraph): the fastest launch period of
# the pattern over every occupancy (waves per CU, by an LDS pad) and VALU count tried -- the ceiling
# the step's own period is compared with (bench.py pattern_ceiling)
rows = []
for name in ("r05_mover_sweep_4m.txt", "r05_mover_occupancy_4m.txt"):
    sweep = os.path.join(root, "profiles", name)
    if not os.path.exists(sweep):
        continue
    for ln in open(sweep):
        if "waves/CU" in ln and "us/launch" in ln:
            occ = ln.split("waves/CU")[1].split()[0]
            rows.append((name, occ, int(ln.split("VALU/lane")[1].split(":")[0]), float(ln.split(":")[1].split("us")[0])))
if rows:
    best = min(rows, key=lambda r: r[3])
    out["period_us_event_timed"] = best[3]
    out["period_source"] = (f"profiles/{best[0]}: the fastest case of the sweeps ({best[1]} waves per CU, {best[2]} VALU "
                            "per lane), HIP events over 100-launch graphs")
    out["ceiling_GBs_315"] = 315 * n / best[3] / 1e3
    out["sweep_cases"] = len(rows)
with open(summary, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "cases"}, indent=1))
