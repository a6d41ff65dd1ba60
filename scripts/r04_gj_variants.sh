# Per-round phase timing of the device trim for library variants (HG_TIMING builds in build/variants).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-timing}; do
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/gj_$v.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/gj_$v.txt; exit 3; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/gj_$v.txt
done
