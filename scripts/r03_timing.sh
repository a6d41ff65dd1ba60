# Phase timing (HG_TIMING builds) of the current kernel and of round 2's, one after the other.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-timing r02_timing}; do
  echo "== $v"
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/timing_probe.py --envs ${N:-65536} > gpurun_out/timing_$v.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/timing_$v.txt; exit 3; }
  cat gpurun_out/timing_$v.txt
done
