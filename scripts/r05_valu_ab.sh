# Round 5: VALU / SALU instructions per wave of the headline kernel on an aged population, per library
# variant (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_WAVES in one --pmc pass), then the interleaved timing A/B.
#   VARIANTS="cur prev att1g1 att0g3"
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"cur prev"}
for v in $VARIANTS; do
  if [ "$v" = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
  D=gpurun_out/valu_$v; rm -rf $D; mkdir -p $D
  HELIGYM_AMD_LIB=$lib timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d $D -o run -- python3 bench.py --steps 200 --warmup 20 --repeats 1 --age-seconds ${PMC_AGE:-60} --no-secondary --no-cpu-baseline --no-parity > $D/log.txt 2>&1 || { echo "pmc $v failed"; tail -5 $D/log.txt; exit 4; }
  python3 - "$D" "$v" <<'PY'
import csv, glob, sys, re
d, v = sys.argv[1], sys.argv[2]
pat = re.compile(r"step_kernel<1, false, true, false, false, true(, false)?>")
agg = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat.search(r.get("Kernel_Name", "")):
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
m = {k: sum(x) / len(x) for k, x in agg.items()}
w = m.get("SQ_WAVES", 1)
print(f"{v:8s} launches {len(agg.get('SQ_WAVES', []))}  VALU/wave {m.get('SQ_INSTS_VALU', 0) / w:7.1f}  SALU/wave {m.get('SQ_INSTS_SALU', 0) / w:6.1f}  SMEM/wave {m.get('SQ_INSTS_SMEM', 0) / w:5.1f}")
PY
  find $D -name "*.csv" -size +2M -delete
done
VARIANTS="$VARIANTS" ROUNDS=${ROUNDS:-3} TAG=${TAG:-valu} bash scripts/ab.sh
