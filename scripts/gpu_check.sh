# GPU round check: parity tests, bench, kernel-trace profile.  Every GPU step has its own time
# limit; a crash/timeout (anything but a test failure) stops the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^\[|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1000 --no-cpu-baseline --no-parity > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 4; }
  find gpurun_out/prof -name "*stats*" | head
  cat $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) | head -12
fi
exit 0
