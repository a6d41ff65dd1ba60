# two-wave vs single-wave specialised kernel: phase timing and issue counters at 65536 envs
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp5
export TMPDIR=/tmp
HELIGYM_AMD_LIB=$PWD/build/variants/TP.so timeout -k 10 120 python scripts/timing_probe.py --pair > gpurun_out/exp5/timing_pair.log 2>&1 || { echo timing pair failed; tail gpurun_out/exp5/timing_pair.log; exit 3; }
HELIGYM_AMD_LIB=$PWD/build/variants/TS.so timeout -k 10 120 python scripts/timing_probe.py > gpurun_out/exp5/timing_single.log 2>&1 || { echo timing single failed; tail gpurun_out/exp5/timing_single.log; exit 3; }
cat gpurun_out/exp5/timing_pair.log gpurun_out/exp5/timing_single.log | grep -v amdgpu.ids
for v in pair NP; do
  lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; [ $v = NP ] && lib=$PWD/build/variants/NP.so
  HELIGYM_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS --output-format csv -d gpurun_out/exp5/$v.a -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-parity --rollout-steps 0 > gpurun_out/exp5/$v.a.log 2>&1 || { echo pmc a $v failed; exit 4; }
  HELIGYM_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/exp5/$v.b -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-parity --rollout-steps 0 > gpurun_out/exp5/$v.b.log 2>&1 || { echo pmc b $v failed; exit 4; }
done
python3 - <<'PY'
import csv, glob, collections
for v in ("pair", "NP"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/exp5/{v}.*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    w = sum(agg["SQ_WAVES"]) / max(1, len(agg["SQ_WAVES"]))
    print(v, "waves/launch", w)
    for k, x in sorted(agg.items()):
        m = sum(x) / len(x)
        print(f"  {k:22s} per launch {m:12.0f}  per wave {m / max(w, 1):10.1f}")
PY
