# Helper kernel (default build) against the one-wave kernel (h0) and the wider threshold (d2):
# GPU tests of the variants file, then interleaved A/B at 4 096 .. 65 536 envs.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/helper_ab2.txt; : > $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_variants.py -m gpu > gpurun_out/helper_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/helper_tests.txt; exit 3; }
tail -3 gpurun_out/helper_tests.txt
for envs in 4096 16384 32768 65536; do
  for r in 1 2 3; do
    for v in cur h0 d2; do
      if [ $v = cur ]; then lib=$PWD/heli-gym_amd/heligym_amd/libheligym_amd.so; else lib=$PWD/build/variants/$v.so; fi
      HELIGYM_AMD_LIB=$lib timeout -k 10 150 python bench.py --envs $envs --steps 1000 --repeats 3 --no-secondary --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1 || { echo "$v failed" | tee -a $O; tail -3 gpurun_out/ab.log; exit 3; }
      echo "envs $envs $v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3, 3))')" | tee -a $O
    done
  done
done
