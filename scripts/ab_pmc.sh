# A/B of the headline bench between the in-tree library (cur) and build/variants/$B.so, interleaved,
# then one PMC pass of instruction / cycle counters per library.  Every GPU step has its own limit.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
N=${N:-65536}
for r in ${RS:-1 2 3}; do
  for v in ${A:-cur} ${B:-r02}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    HELIGYM_AMD_LIB=$lib timeout -k 10 120 python bench.py --envs $N --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab.log; exit 3; }
    echo "$v N=$N $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))') us"
  done
done
if [ "${PMC:-1}" = "1" ]; then
  for v in ${A:-cur} ${B:-r02}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    i=0
    for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
               "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      HELIGYM_AMD_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_${v}_$N/p$i -o run -- python3 bench.py --envs $N --steps 200 --warmup 20 --repeats 1 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/pmc_${v}_$N.log 2>&1 || { echo "pmc $v $i failed"; tail -5 gpurun_out/pmc_${v}_$N.log; exit 4; }
    done
  done
  python3 scripts/pmc_brief.py gpurun_out ${A:-cur} ${B:-r02} $N
fi
