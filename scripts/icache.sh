# instruction-cache counters of the step kernel per library variant (VARIANTS), one --pmc pass each
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ic
export TMPDIR=/tmp
for v in ${VARIANTS:-H0 H1}; do
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d gpurun_out/ic/$v -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-parity --rollout-steps 0 > gpurun_out/ic/$v.log 2>&1 || { echo "pmc $v failed"; exit 3; }
done
python3 - <<'PY'
import csv, glob, collections, os
for v in os.environ.get("VARIANTS", "H0 H1").split():
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/ic/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "false, true>" in r.get("Kernel_Name", "") and "step_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in agg.items()})
PY
