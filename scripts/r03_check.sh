# Round-3 GPU check: pytest -m gpu (per-test time limit), then the default bench line.
# Every GPU step has its own limit; anything but a plain test failure stops the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -20
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu.log; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log
fi
exit 0
