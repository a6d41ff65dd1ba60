set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python scripts/r04_gj_ab.py base > gpurun_out/gj_ab_base.txt 2>&1 || { echo "ab base failed"; tail -5 gpurun_out/gj_ab_base.txt; exit 3; }
HELIGYM_AMD_LIB=$PWD/build/variants/gjsplit.so timeout -k 10 120 python scripts/r04_gj_ab.py split > gpurun_out/gj_ab_split.txt 2>&1 || { echo "ab split failed"; tail -5 gpurun_out/gj_ab_split.txt; exit 3; }
grep -h "\[" gpurun_out/gj_ab_base.txt gpurun_out/gj_ab_split.txt
python -c "
import numpy as np
a=np.load('gpurun_out/gj_base.npz'); b=np.load('gpurun_out/gj_split.npz')
print('bitwise', all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files), 'status ok', int((a['status']==0).sum()))"
bash scripts/r04_check.sh
