# Round-4: landing-gear forms -- per point (gear0), moment factored (gear2), fully factored (default):
# headline step time and the through-contact parity margins.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in default gear2 gear0; do
  lib=""; [ $v != default ] && lib=$PWD/build/variants/$v.so
  HELIGYM_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "through_contact or single_step_vs_oracle" > gpurun_out/gm_$v.txt 2>&1
  echo "== $v"; grep -h "^\[contact\|^\[oracle\|passed\|failed" gpurun_out/gm_$v.txt
  HELIGYM_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-parity > gpurun_out/gb_$v.log 2>&1 || { echo "bench failed"; exit 4; }
  tail -1 gpurun_out/gb_$v.log > gpurun_out/gb_$v.json; python scripts/bench_brief.py gpurun_out/gb_$v.json | head -1
done
