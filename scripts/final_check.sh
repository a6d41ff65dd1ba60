# End-of-round confirmation on the GPU box: pytest -m gpu + smoke(), the default bench line with a
# rocprofv3 kernel trace of the same command, the BASELINE config sweep and the re-trim phase timing
# (HG_TIMING build in build/variants/timing.so).  Every GPU step has its own limit; stop on a crash.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 > gpurun_out/final_gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/final_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/final_gpu_tests.txt 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/final_gpu_tests.txt; exit 3; }
tail -1 gpurun_out/final_gpu_tests.txt
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/final_bench.log; exit 4; }
tail -1 gpurun_out/final_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o bench -- python3 bench.py --no-cpu-baseline --no-parity > gpurun_out/final_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/final_prof.log; exit 5; }
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/retrim_timing.txt 2>&1 || { echo "retrim timing failed"; exit 6; }
bash scripts/bench_sweep.sh
