# Interleaved A/B of the headline bench between the in-tree library and build/variants/$B.so
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in cur ${B:-prev}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    HELIGYM_AMD_LIB=$lib timeout -k 10 120 python bench.py --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab.log; exit 3; }
    echo "$v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))')"
  done
done
