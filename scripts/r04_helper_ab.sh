# Wind helper waves (HG_HELPER): bitwise against the in-tree library, then interleaved A/B of the
# headline (65 536 envs) and config 2 (4 096 envs) against it.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/helper_ab.txt; : > $O
for v in cur ${VARS:-h1 h2 h4}; do
  if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
  for cfg in "65536 300" "4100 300"; do
    HELIGYM_AMD_LIB=$lib timeout -k 10 120 python -u scripts/r04_helper_bits.py $cfg >> $O 2>&1 || { echo "$v bits failed" | tee -a $O; tail -5 $O; exit 3; }
  done
  tail -2 $O
done
for envs in 65536 4096; do
  for r in 1 2 3; do
    for v in cur ${VARS:-h1 h2 h4}; do
      if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
      HELIGYM_AMD_LIB=$lib timeout -k 10 150 python bench.py --envs $envs --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed" | tee -a $O; tail -3 gpurun_out/ab.log; exit 3; }
      echo "envs $envs $v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))')" | tee -a $O
    done
  done
done
