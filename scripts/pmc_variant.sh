# Issue/stall counters of the step kernel for library variants (diagnostic; gpurun_out only)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcv
export TMPDIR=/tmp
for v in ${VARIANTS:-N}; do for n in ${SIZES:-65536 1048576}; do
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
    tag=$(echo $set | cut -c1-12 | tr ' ' '_')
    HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmcv/${v}_${n}_$tag -o run -- python3 bench.py --envs $n --steps 100 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/pmcv/${v}_${n}_$tag.log 2>&1 || { echo "pmc $v $n failed"; tail -5 gpurun_out/pmcv/${v}_${n}_$tag.log; exit 3; }
  done
done; done
python3 - <<'PY'
import csv, glob, collections, os
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcv/*/run_counter_collection.csv"):
    key = "_".join(os.path.basename(os.path.dirname(f)).split("_")[:2])
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r.get("Kernel_Name", ""):
            res[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(res):
    m = {k: sum(v)/len(v) for k, v in res[key].items()}
    w = m.get("SQ_WAVES", 1)
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(key, " ".join(f"{k[3:]}={m[k]/w:.0f}/wave" for k in ("SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_INSTS_SMEM","SQ_INSTS_BRANCH") if k in m),
          f"wave_cyc={wc/w:.0f}q", " ".join(f"{k[3:]}={100*m[k]/wc:.0f}%" for k in ("SQ_WAIT_ANY","SQ_WAIT_INST_ANY","SQ_ACTIVE_INST_ANY","SQ_ACTIVE_INST_VALU","SQ_ACTIVE_INST_SCA") if k in m),
          f"busy={m.get('SQ_BUSY_CYCLES',0):.0f}")
PY
