# Round 5: re-trim solve variants (retrim_body.h HG_GJ_SPEC, HG_RT_XLDS).  Phase timing of one trim per
# HG_TIMING build (TV, build/variants/<name>.so), then the interleaved A/B of the bench's re-trim
# secondaries (AV: cur = the in-tree library, others build/variants/<name>.so).
#   TV="tcur tspec1 tnoxlds" AV="cur spec1 noxlds" TAG=spec bash scripts/r05_spec.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${TV:-tcur tspec1 tnoxlds}; do
  echo "== $v"
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/rt_$v.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/rt_$v.txt; exit 3; }
  grep -v amdgpu.ids gpurun_out/rt_$v.txt
done
VARIANTS="${AV:-cur spec1 noxlds}" ROUNDS=${ROUNDS:-2} TAG=${TAG:-spec} FIELD=retrim.ms_per_step \
  ARGS="--steps 500 --repeats 3 --no-cpu-baseline --no-parity" bash scripts/ab.sh || exit 4
python3 - gpurun_out/ab_${TAG:-spec}.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    print(d["variant"], d["ab_round"], "step", round(d["ms_per_step"] * 1e3, 3), "retrim", round(d["retrim"]["ms_per_step"] * 1e3, 2),
          "next", round(d.get("retrim_next_step", {}).get("ms_per_step", float("nan")) * 1e3, 2))
PY
