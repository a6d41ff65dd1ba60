# Round-4 probes: HIP timing events inside a hipGraph (short bench windows), the re-trim phase timing
# of the Gauss-Jordan variants (HG_TIMING builds) and an A/B of the replicated-column solve.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python scripts/r04_inner_events.py > gpurun_out/inner_events.txt 2>&1
grep -v amdgpu.ids gpurun_out/inner_events.txt | tail -6
VARIANTS="tbase tsplit tsplit2" bash scripts/r04_gj_variants.sh || exit 3
timeout -k 10 120 python scripts/r04_gj_ab.py base > gpurun_out/gj_ab_base.txt 2>&1 || { echo "ab base failed"; exit 4; }
HELIGYM_AMD_LIB=$PWD/build/variants/gjsplit2.so timeout -k 10 120 python scripts/r04_gj_ab.py split2 > gpurun_out/gj_ab_split2.txt 2>&1 || { echo "ab split2 failed"; tail -3 gpurun_out/gj_ab_split2.txt; exit 5; }
grep -h "\[" gpurun_out/gj_ab_base.txt gpurun_out/gj_ab_split2.txt
python -c "
import numpy as np
a=np.load('gpurun_out/gj_base.npz'); b=np.load('gpurun_out/gj_split2.npz')
print('bitwise', all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files))"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b20.log 2>&1 || { echo "bench 20 failed"; grep -v "^frame" gpurun_out/b20.log | tail -8; exit 6; }
tail -1 gpurun_out/b20.log > gpurun_out/b20.json; python scripts/bench_brief.py gpurun_out/b20.json
