# GPU tests, then specialised vs generic kernel at several batch sizes (one bench process per point)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
out=gpurun_out/ab.jsonl; : > $out
run() { timeout -k 10 200 python bench.py --steps 1000 --no-cpu-baseline --no-parity "$@" | python -c "import sys,json; d=json.loads(sys.stdin.read()); d['args']='${LABEL:-} $*'; print(json.dumps(d))" >> $out || { echo "bench $* failed"; exit 3; }; }
for n in ${SIZES:-65536 262144 1048576}; do
  run --envs $n
  [ "${GENERIC:-1}" = "1" ] && run --envs $n --generic-kernel
done
python - <<'PY'
import json
for l in open("gpurun_out/ab.jsonl"):
    d = json.loads(l); r = d["roofline"]; ro = d.get("rollout") or {}
    print(f'{d["args"]:40s} {d["value"]:.3e} steps/s {d["ms_per_step"]*1e3:7.2f} us/step frac {r["frac"]:.3f} | rollout {ro.get("ms_per_step", 0)*1e3:6.2f} us/step')
PY
