# Round-4 confirmation on the GPU box: pytest -m gpu + smoke(), the bench line at the default 1 000
# steps and at the driver's short window, the kernel trace of the headline command, PMC passes at
# 65 536 and 4 M envs, the BASELINE config sweep and the re-trim phase timing.  Each GPU step has its own
# time limit; a crash or timeout stops the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "[final] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/final_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/final_gpu_tests.txt 2>&1 || { echo "smoke failed"; exit 3; }
tail -1 gpurun_out/final_gpu_tests.txt
echo "[final] bench"
timeout -k 10 500 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/final_bench.log; exit 4; }
tail -1 gpurun_out/final_bench.log > gpurun_out/final_bench.json; python scripts/bench_brief.py gpurun_out/final_bench.json
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_short.log 2>&1 || { echo "short bench failed"; tail -5 gpurun_out/final_bench_short.log; exit 5; }
tail -1 gpurun_out/final_bench_short.log > gpurun_out/final_bench_short.json; python scripts/bench_brief.py gpurun_out/final_bench_short.json | head -1
echo "[final] trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o bench -- python3 bench.py --no-cpu-baseline --no-parity --no-secondary > gpurun_out/final_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/final_prof.log; exit 6; }
tail -1 gpurun_out/final_prof.log > gpurun_out/final_prof_line.json
find gpurun_out/final_prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo "[final] pmc"
TAG=r04c N=65536 bash scripts/profile_round.sh || exit 7
TAG=r04d N=4194304 TRACE_STEPS=200 bash scripts/profile_round.sh || exit 8
echo "[final] sweep"
bash scripts/bench_sweep.sh || exit 9
echo "[final] re-trim timing"
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/final_retrim_timing.txt 2>&1 || { echo "retrim timing failed"; exit 10; }
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/timing_probe.py --warm 6000 > gpurun_out/final_phase_timing.txt 2>&1 || { echo "phase timing failed"; exit 11; }
grep -v amdgpu.ids gpurun_out/final_retrim_timing.txt | head -3; grep -h "wave life\|branch flags" gpurun_out/final_phase_timing.txt
echo "[final] done"
