# Round-4: the re-trim residual taken from the LDS hand-off (no per-round scalar loads of y*, no
# single-lane writes): trims bitwise against the previous library, step times, re-trim tests, phase timing.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in prev default; do
  lib=""; [ $v != default ] && lib=$PWD/build/variants/$v.so
  HELIGYM_AMD_LIB=$lib timeout -k 10 120 python scripts/r04_gj_ab.py $v > gpurun_out/gj_ab_$v.txt 2>&1 || { echo "ab $v failed"; tail -3 gpurun_out/gj_ab_$v.txt; exit 3; }
  grep -h "\[" gpurun_out/gj_ab_$v.txt
done
python -c "
import numpy as np
a=np.load('gpurun_out/gj_prev.npz'); b=np.load('gpurun_out/gj_default.npz')
print('bitwise', all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files))"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "trim or retrim or overlap or reset or azimuth or single_env" > gpurun_out/rt_tests.txt 2>&1; tail -2 gpurun_out/rt_tests.txt
VARIANTS="timing" bash scripts/r04_gj_variants.sh
