# Issue microbenchmark, then A/B of the headline (65 536) and the out-of-cache (4 M envs) step
# between the in-tree library and variants.  Each GPU step has its own limit.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${DEP:-1}" = 1 ] && [ -x build/dep ]; then timeout -k 10 60 ./build/dep | tee gpurun_out/dep.txt || exit 3; fi
for N in ${NS:-65536 4194304}; do
  for r in 1 2; do
    for v in cur ${VARIANTS:-r02}; do
      if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
      st=1000; [ $N -gt 1000000 ] && st=200
      HELIGYM_AMD_LIB=$lib timeout -k 10 180 python bench.py --envs $N --steps $st --repeats 3 --warmup 20 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab.log; exit 3; }
      echo "$v N=$N $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))') us"
    done
  done
done
