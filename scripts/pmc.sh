# Hardware counters for the step kernel (separate --pmc passes, kernel-trace only, no sys/runtime trace)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
N=${N:-65536}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --envs $N --steps 200 --warmup 20 --no-cpu-baseline --no-parity > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/pmc/p$i.log; exit 3; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:24s} n={len(v):5d} mean={sum(v)/len(v):.4g}")
PY
