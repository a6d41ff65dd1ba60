# Round 5: re-trim variants (retrim_body.h HG_RT_XLDS, HG_RT_VLOAD; the dropped HG_GJ_SPEC, prefetch).  Phase timing of one trim per
# HG_TIMING build (TV, build/variants/<name>.so), then the interleaved A/B of the bench's re-trim
# secondaries (AV: cur = the in-tree library, others build/variants/<name>.so).
#   TV="tcur tnovl" AV="cur novl" TAG=vl bash scripts/r05_spec.sh   (variants: scripts/build_variants.py)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${TV:-tcur tnovl}; do
  echo "== $v"
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/rt_$v.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/rt_$v.txt; exit 3; }
  grep -v amdgpu.ids gpurun_out/rt_$v.txt
done
VARIANTS="${AV:-cur novl}" ROUNDS=${ROUNDS:-2} TAG=${TAG:-spec} FIELD=retrim.ms_per_step \
  ARGS="--steps 500 --repeats 3 --no-cpu-baseline --no-parity" bash scripts/ab.sh || exit 4
python3 - gpurun_out/ab_${TAG:-spec}.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    print(d["variant"], d["ab_round"], "step", round(d["ms_per_step"] * 1e3, 3), "retrim", round(d["retrim"]["ms_per_step"] * 1e3, 2),
          "next", round(d.get("retrim_next_step", {}).get("ms_per_step", float("nan")) * 1e3, 2))
PY
