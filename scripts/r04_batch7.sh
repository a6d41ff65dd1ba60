# Round-4: re-trim evaluation rows padded to 17 doubles in LDS (bank conflicts of the hand-off):
# phase timing (HG_TIMING builds t16 / t17), trims bitwise against the 16-double layout (e16), and
# the re-trim step times.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS="t16 t17" bash scripts/r04_gj_variants.sh || exit 3
HELIGYM_AMD_LIB=$PWD/build/variants/e16.so timeout -k 10 120 python scripts/r04_gj_ab.py e16 > gpurun_out/gj_ab_e16.txt 2>&1 || { echo "ab e16 failed"; exit 4; }
timeout -k 10 120 python scripts/r04_gj_ab.py e17 > gpurun_out/gj_ab_e17.txt 2>&1 || { echo "ab e17 failed"; exit 5; }
grep -h "\[" gpurun_out/gj_ab_e16.txt gpurun_out/gj_ab_e17.txt
python -c "
import numpy as np
a=np.load('gpurun_out/gj_e16.npz'); b=np.load('gpurun_out/gj_e17.npz')
print('bitwise', all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files))"
