# Bulk-launch occupancy A/B (two waves per SIMD via the LDS cap vs three) at 262 144 FF, 1 M and 4 M
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for v in cur ${VARIANTS:-nocap r02}; do
    if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
    for cfg in "--envs 262144 --task forward_flight --steps 500" "--envs 1048576 --steps 300" "--envs 4194304 --steps 200"; do
      HELIGYM_AMD_LIB=$lib timeout -k 10 180 python bench.py $cfg --repeats 3 --warmup 20 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/occ.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/occ.log; exit 3; }
      echo "$v $cfg $(tail -1 gpurun_out/occ.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 2))') us"
    done
  done
done
