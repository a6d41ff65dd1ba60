# Interleaved A/B of the re-trim step (bench.py's retrim secondary, graph-replayed, 65 536 envs) between
# the in-tree library and build/variants/$B.so
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in cur ${B:-gj0}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    HELIGYM_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 500 --repeats 3 --no-cpu-baseline --no-parity > gpurun_out/abr.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abr.log; exit 3; }
    echo "$v $(tail -1 gpurun_out/abr.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step", round(d["ms_per_step"]*1e3, 3), "retrim", round(d["retrim"]["ms_per_step"]*1e3, 2), "fail", d["retrim"]["retrim_failures"])')"
  done
done
