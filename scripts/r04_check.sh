# Round-4 GPU check: pytest -m gpu + smoke(), then the bench line twice -- the default 1 000-step
# windows and the driver's short run (--steps 20 --warmup 5) -- both on aged populations.  Every GPU
# step has its own limit; a crash or timeout stops the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.txt 2>&1
  rc=$?; tail -3 gpurun_out/r04_gpu_tests.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r04_gpu_tests.txt 2>&1 || { echo "smoke failed"; exit 3; }
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/r04_bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r04_bench_default.log; exit 4; }
tail -1 gpurun_out/r04_bench_default.log > gpurun_out/r04_bench_default.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/r04_bench_short.log 2>&1 || { echo "short bench failed"; tail -5 gpurun_out/r04_bench_short.log; exit 5; }
tail -1 gpurun_out/r04_bench_short.log > gpurun_out/r04_bench_short.json
python scripts/bench_brief.py gpurun_out/r04_bench_default.json gpurun_out/r04_bench_short.json
