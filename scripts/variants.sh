# A/B the library variants under build/variants (each bench in its own process and time limit)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/variants.jsonl; : > $out
for v in ${VARIANTS:-A B C D}; do
  for n in ${SIZES:-65536 1048576}; do
    HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 200 python bench.py --envs $n --steps 1000 --no-cpu-baseline \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> $out \
      || { echo "variant $v failed"; exit 3; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/variants.jsonl"):
    d = json.loads(l); r = d["roofline"]; p = d.get("max_abs_step_err") or {}
    ro = d.get("rollout") or {}
    print(f'{d["variant"]} N={d["config"]["envs_per_gpu"]:8d} {d["value"]:.3e} steps/s {d["ms_per_step"]*1e3:7.1f} us/step kern {r["kernel_avg_us"]:7.1f} us frac {r["frac"]:.3f} err/tol {p.get("max_err_over_tol", -1):.3f}'
          f' | rollout {ro.get("value", 0):.3e} steps/s {ro.get("ms_per_step", 0)*1e3:6.1f} us/step')
PY
