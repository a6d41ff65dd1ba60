# phase timing of timing-build variants (TIMING="TA TB ..."), then A/B benches (VARIANTS="...")
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${TIMING:-TA}; do
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/timing_probe.py > gpurun_out/timing_$v.log 2>&1 || { echo timing $v failed; tail gpurun_out/timing_$v.log; exit 3; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/timing_$v.log
done
[ -n "${VARIANTS:-}" ] && bash scripts/variants.sh
exit 0
