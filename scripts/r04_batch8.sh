# Round-4: the factored landing-gear loads -- the GPU parity suite (contact trajectories included), then
# headline and 4 M-env steps against the per-point form (gear0), aged 60 s.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r04_gpu_tests.txt; grep -h "max\|FAIL\|Error" gpurun_out/r04_gpu_tests.txt | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/b_$tag.log 2>&1 || { echo "bench $tag failed"; grep -v "^frame" gpurun_out/b_$tag.log | tail -6; exit 4; }
  tail -1 gpurun_out/b_$tag.log > gpurun_out/b_$tag.json; python scripts/bench_brief.py gpurun_out/b_$tag.json | head -1
}
for r in 1 2; do
  run fac$r --no-secondary --no-cpu-baseline --no-parity
  HELIGYM_AMD_LIB=$PWD/build/variants/gear0.so run gear0_$r --no-secondary --no-cpu-baseline --no-parity
done
run fac4m --envs 4194304 --steps 200 --repeats 3 --no-secondary --no-cpu-baseline --no-parity
HELIGYM_AMD_LIB=$PWD/build/variants/gear0.so run gear0_4m --envs 4194304 --steps 200 --repeats 3 --no-secondary --no-cpu-baseline --no-parity
run fac_parity --steps 20 --no-secondary --no-cpu-baseline
python -c "import json; d=json.load(open('gpurun_out/b_fac_parity.json')); print('max_abs_step_err', d.get('max_abs_step_err'))"
