# Round-4: the aged population (branch shares by age), and the bench windows aged 60 s: TimedGraph
# (events inside the graph) at K = 20 and 1 000 against the graph-replay windows at K = 20.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/r04_population.py > gpurun_out/population.txt 2>&1 || { echo "population failed"; tail -5 gpurun_out/population.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/population.txt
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/b_$tag.log 2>&1 || { echo "bench $tag failed"; grep -v "^frame" gpurun_out/b_$tag.log | tail -6; exit 4; }
  tail -1 gpurun_out/b_$tag.log > gpurun_out/b_$tag.json; python scripts/bench_brief.py gpurun_out/b_$tag.json
}
run k20 --steps 20 --warmup 5 --age-seconds 60 --no-cpu-baseline
HG_BENCH_OUTER_WINDOWS=1 run k20outer --steps 20 --warmup 5 --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
run k1000 --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
HG_BENCH_OUTER_WINDOWS=1 run k1000outer --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
# the medium-angle series (default) against the full sincos past 0.05 rad (nomid), aged 60 s, K = 1 000
HELIGYM_AMD_LIB=$PWD/build/variants/nomid.so run nomid --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
HELIGYM_AMD_LIB=$PWD/build/variants/nomid.so run nomid4m --envs 4194304 --steps 200 --repeats 3 --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
run mid4m --envs 4194304 --steps 200 --repeats 3 --age-seconds 60 --no-secondary --no-cpu-baseline --no-parity
HELIGYM_AMD_LIB=$PWD/build/variants/tmid.so timeout -k 10 120 python scripts/timing_probe.py --warm 6000 > gpurun_out/phase_timing_mid.txt 2>&1 || { echo "timing failed"; exit 5; }
grep -h "wave life\|branch flags\|waves:" gpurun_out/phase_timing_mid.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/r04_gpu_tests.txt; exit $rc
