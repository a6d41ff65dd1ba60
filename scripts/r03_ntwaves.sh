set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for v in cur ${VARIANTS:-nt3 nt1}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    for n in ${NS:-196608 262144}; do
      HELIGYM_AMD_LIB=$lib timeout -k 10 180 python bench.py --envs $n --steps 500 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/nt.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/nt.log; exit 3; }
      echo "$v N=$n $(tail -1 gpurun_out/nt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))') us"
    done
  done
done
