# Round-4: re-trim trial points formed with one select per component, and the device fp64 sqrt
# (rsq + Goldschmidt): trims bitwise against the previous library for the first change alone
# (sqrtlibm), step times (prev / new), the re-trim parity tests and phase timing.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in prev sqrtlibm default; do
  lib=""; [ $v != default ] && lib=$PWD/build/variants/$v.so
  HELIGYM_AMD_LIB=$lib timeout -k 10 120 python scripts/r04_gj_ab.py $v > gpurun_out/gj_ab_$v.txt 2>&1 || { echo "ab $v failed"; tail -3 gpurun_out/gj_ab_$v.txt; exit 3; }
  grep -h "\[" gpurun_out/gj_ab_$v.txt
done
python -c "
import numpy as np
a=np.load('gpurun_out/gj_prev.npz'); b=np.load('gpurun_out/gj_sqrtlibm.npz'); c=np.load('gpurun_out/gj_default.npz')
print('trial points alone bitwise', all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files))
d=np.abs(a['state'].astype(np.float64)-c['state']); print('fast sqrt: max |d state|', d.max(), 'rel', (d/np.maximum(np.abs(a['state']),1e-6)).max(), 'status equal', np.array_equal(a['status'], c['status']))"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "trim or retrim or overlap or reset or azimuth or single_env" > gpurun_out/rt_tests.txt 2>&1; tail -2 gpurun_out/rt_tests.txt
VARIANTS="tnew" bash scripts/r04_gj_variants.sh
