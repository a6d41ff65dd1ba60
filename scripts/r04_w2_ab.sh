# Stage 1's wind-independent part (kinematics, gear) formed before the helper hand-over (cur) against
# the helper kernel without it (prev): digests, the variants tests, then interleaved A/B.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/w2_ab.txt; : > $O
for v in cur w2; do
  if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
  for cfg in "65536 300" "4100 300"; do
    HELIGYM_AMD_LIB=$lib timeout -k 10 120 python -u scripts/r04_helper_bits.py $cfg 2>&1 | grep digest >> $O || { echo "$v bits failed" | tee -a $O; exit 3; }
  done
done
cat $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_variants.py -m gpu > gpurun_out/w2_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pre_tests.txt; exit 3; }
tail -1 gpurun_out/w2_tests.txt
for envs in 4096 32768 65536; do
  for r in 1 2 3; do
    for v in cur w2; do
      if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
      HELIGYM_AMD_LIB=$lib timeout -k 10 150 python bench.py --envs $envs --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed" | tee -a $O; tail -3 gpurun_out/ab.log; exit 3; }
      echo "envs $envs $v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))')" | tee -a $O
    done
  done
done
