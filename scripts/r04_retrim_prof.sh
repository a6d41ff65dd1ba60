# Re-trim kernel trace: the bench with reset_mode "retrim" as the headline (aged), under rocprofv3
# --kernel-trace --stats; then the phase timing of the HG_TIMING build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-trim or retrim or azimuth}" > gpurun_out/r04_retrim_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04_retrim_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/r04_retrim_timing.txt 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r04_retrim_timing.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r04_retrim_timing.txt
rm -rf gpurun_out/prof_rt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rt -o rt -- python3 bench.py --reset-mode retrim ${BENCH_ARGS:---autoreset-mode same_step} --no-secondary --steps 200 --no-cpu-baseline --no-parity > gpurun_out/r04_prof_rt.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r04_prof_rt.log; exit 4; }
tail -1 gpurun_out/r04_prof_rt.log | cut -c1-400
f=$(find gpurun_out/prof_rt -name "*kernel_stats.csv" | head -1); head -6 "$f" | cut -d, -f1-8
for v in ${AB:-}; do
  HELIGYM_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 200 python bench.py --reset-mode retrim --no-secondary --steps 200 --no-cpu-baseline --no-parity > gpurun_out/r04_ab_$v.log 2>&1 || { echo "ab $v failed"; exit 6; }
  echo "$v: $(tail -1 gpurun_out/r04_ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1e3, d["timing"]["resets_in_window"])')"
done
timeout -k 10 200 python bench.py --reset-mode retrim --no-secondary --steps 200 --no-cpu-baseline --no-parity > gpurun_out/r04_ab_default.log 2>&1 || exit 7
echo "default: $(tail -1 gpurun_out/r04_ab_default.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1e3, d["timing"]["resets_in_window"])')"
